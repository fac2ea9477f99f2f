"""slm_copy_bandwidth: the measured streaming-copy rate bench.py reports next
to the 8 TB/s spec ("a measured copy-kernel peak")."""
import pytest


@pytest.mark.gpu
def test_copy_bandwidth_is_plausible(gpu):
    hbm = gpu.copy_bandwidth(1 << 28, 5)
    small = gpu.copy_bandwidth(10 << 20, 20)
    print(f"[bandwidth] copy 256 MiB buffers {hbm:.0f} GB/s, 10 MiB buffers {small:.0f} GB/s")
    assert 1000.0 < hbm < 12000.0
    assert 500.0 < small < 40000.0


@pytest.mark.gpu
def test_copy_bandwidth_rejects_bad_arguments(gpu):
    with pytest.raises(gpu.SlmError):
        gpu.copy_bandwidth(8, 1)
    with pytest.raises(gpu.SlmError):
        gpu.copy_bandwidth(1 << 20, 0)
