// Instantiates the complex128 radix-plan kernels (radix_c128.hpp) of one plan
// key SLM_N, like kernels_inst.hip for the float32 engine: one object per key
// (Makefile), so the builds run in parallel.
#include "radix_c128.hpp"

#ifndef SLM_N
#error "compile with -DSLM_N=<plan key>"
#endif

#define SLM_PASTE2(a, b) a##b
#define SLM_PASTE(a, b) SLM_PASTE2(a, b)

namespace slm {
namespace rz {
namespace {

static_assert(key_built(SLM_N), "plan key without complex128 kernels");

template <int OP, int LAY>
int row_one(const mr::RowArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL((rz_row_kernel<SLM_N, OP, LAY>), dim3(grid), dim3(RowGeo<SLM_N, LAY>::THREADS), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int CW, int OP, int LAY>
int col_one(const mr::ColArgs& a, int grid, hipStream_t st) {
    if constexpr (!ColGeo<SLM_N, CW>::kValid) {
        return -1;
    } else {
        hipLaunchKernelGGL((rz_col_kernel<SLM_N, CW, OP, LAY>), dim3(grid), dim3(ColGeo<SLM_N, CW>::THREADS), 0, st,
                           a);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
}

template <int CW, int LAY>
int col_cw(int op, const mr::ColArgs& a, int grid, hipStream_t st) {
    using namespace mr;
    switch (op) {
        case CO_FWD: return col_one<CW, CO_FWD, LAY>(a, grid, st);
        case CO_INV: return col_one<CW, CO_INV, LAY>(a, grid, st);
        case CO_AMP_INV: return col_one<CW, CO_AMP_INV, LAY>(a, grid, st);
        case CO_GS: return col_one<CW, CO_GS, LAY>(a, grid, st);
        case CO_GD_STATS: return col_one<CW, CO_GD_STATS, LAY>(a, grid, st);
        case CO_GD_GRAD: return col_one<CW, CO_GD_GRAD, LAY>(a, grid, st);
        case CO_GD_GRAD_U8: return col_one<CW, CO_GD_GRAD_U8, LAY>(a, grid, st);
        default: return -1;
    }
}

template <int LAY>
int row_lay(int op, const mr::RowArgs& a, int grid, hipStream_t st) {
    using namespace mr;
    switch (op) {
        case RO_FWD: return row_one<RO_FWD, LAY>(a, grid, st);
        case RO_INV: return row_one<RO_INV, LAY>(a, grid, st);
        case RO_COLD: return row_one<RO_COLD, LAY>(a, grid, st);
        case RO_WARM: return row_one<RO_WARM, LAY>(a, grid, st);
        case RO_GS: return row_one<RO_GS, LAY>(a, grid, st);
        case RO_GD_FOURIER: return row_one<RO_GD_FOURIER, LAY>(a, grid, st);
        case RO_GD_INIT: return row_one<RO_GD_INIT, LAY>(a, grid, st);
        case RO_GD: return row_one<RO_GD, LAY>(a, grid, st);
        case RO_GS_MID: return row_one<RO_GS_MID, LAY>(a, grid, st);
        default: return -1;
    }
}

template <int LAY>
int col_lay(int cw, int op, const mr::ColArgs& a, int grid, hipStream_t st) {
    switch (cw) {
        case 1: return col_cw<1, LAY>(op, a, grid, st);
        case 2: return col_cw<2, LAY>(op, a, grid, st);
        case 4: return col_cw<4, LAY>(op, a, grid, st);
        case 8: return col_cw<8, LAY>(op, a, grid, st);
        default: return -1;
    }
}

}  // namespace

int SLM_PASTE(rz_row_launch_, SLM_N)(int lay, int op, const mr::RowArgs& a, int grid, hipStream_t st) {
    return lay == LAY_B2 ? row_lay<LAY_B2>(op, a, grid, st) : row_lay<LAY_RM>(op, a, grid, st);
}

int SLM_PASTE(rz_col_launch_, SLM_N)(int lay, int cw, int op, const mr::ColArgs& a, int grid, hipStream_t st) {
    return lay == LAY_B2 ? col_lay<LAY_B2>(cw, op, a, grid, st) : col_lay<LAY_RM>(cw, op, a, grid, st);
}

int SLM_PASTE(rz_row_rpw_, SLM_N)(int lay) {
    return lay == LAY_B2 ? RowGeo<SLM_N, LAY_B2>::RPW : RowGeo<SLM_N, LAY_RM>::RPW;
}

int SLM_PASTE(rz_col_ok_, SLM_N)(int cw) {
    switch (cw) {
        case 1: return ColGeo<SLM_N, 1>::kValid;
        case 2: return ColGeo<SLM_N, 2>::kValid;
        case 4: return ColGeo<SLM_N, 4>::kValid;
        case 8: return ColGeo<SLM_N, 8>::kValid;
        default: return 0;
    }
}

}  // namespace rz
}  // namespace slm
