"""Experimental-setup constants used by the CLI (values of src/constants.py:5-10)."""

slm_width = 1024  # pixels
slm_height = 768  # pixels
wavelength = 5.32e-7  # meters
px_distance = 3.6e-5  # distance between slm pixels in meters
first_diff_max = wavelength / px_distance
u = first_diff_max / 4  # unit convenient for deflecting
