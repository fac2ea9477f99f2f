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

static_assert(key_built(SLM_N, PREC_F64) || key_built(SLM_N, PREC_F32), "plan key without radix kernels");
constexpr bool kF64 = key_built(SLM_N, PREC_F64), kF32 = key_built(SLM_N, PREC_F32);
constexpr bool kPanel = key_panel(SLM_N);  // panel keys: B2 only at either precision

// the complex64 kernels run GS only (generic.hip rz_shape) on 2- and 4-column tiles (rz_cw_of)
template <int P>
constexpr bool row_op_built(int op) {
    return P == PREC_F64 || !(op == mr::RO_GD_FOURIER || op == mr::RO_GD_INIT || op == mr::RO_GD);
}
// (panel keys at float64: 2- and 4-column tiles, every op)
template <int P>
constexpr bool col_op_built(int op, int cw) {
    if constexpr (P == PREC_F64) return !key_panel(SLM_N) || cw == 2 || cw == 4;
    return (cw == 2 || cw == 4) && !(op == mr::CO_GD_STATS || op == mr::CO_GD_GRAD || op == mr::CO_GD_GRAD_U8);
}

template <int CW, int OP, int LAY, int P>
int col_one(const mr::ColArgs& a, int grid, hipStream_t st) {
    if constexpr (!ColGeo<SLM_N, CW, P>::kValid || !col_op_built<P>(OP, CW)) {
        return -1;
    } else {
        hipLaunchKernelGGL((rz_col_kernel<SLM_N, CW, OP, LAY, P>), dim3(grid), dim3(ColGeo<SLM_N, CW, P>::THREADS), 0,
                           st, a);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
}

template <int OP, int LAY, int P>
int row_one(const mr::RowArgs& a, int grid, hipStream_t st) {
    if constexpr (!row_op_built<P>(OP)) {
        return -1;
    } else {
        hipLaunchKernelGGL((rz_row_kernel<SLM_N, OP, LAY, P>), dim3(grid), dim3(RowGeo<SLM_N, LAY>::THREADS), 0, st, a);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
}

template <int CW, int LAY, int P>
int col_cw(int op, const mr::ColArgs& a, int grid, hipStream_t st) {
    using namespace mr;
    switch (op) {
        case CO_FWD: return col_one<CW, CO_FWD, LAY, P>(a, grid, st);
        case CO_INV: return col_one<CW, CO_INV, LAY, P>(a, grid, st);
        case CO_AMP_INV: return col_one<CW, CO_AMP_INV, LAY, P>(a, grid, st);
        case CO_GS: return col_one<CW, CO_GS, LAY, P>(a, grid, st);
        case CO_GD_STATS: return col_one<CW, CO_GD_STATS, LAY, P>(a, grid, st);
        case CO_GD_GRAD: return col_one<CW, CO_GD_GRAD, LAY, P>(a, grid, st);
        case CO_GD_GRAD_U8: return col_one<CW, CO_GD_GRAD_U8, LAY, P>(a, grid, st);
        default: return -1;
    }
}

template <int LAY, int P>
int row_lay(int op, const mr::RowArgs& a, int grid, hipStream_t st) {
    using namespace mr;
    switch (op) {
        case RO_FWD: return row_one<RO_FWD, LAY, P>(a, grid, st);
        case RO_INV: return row_one<RO_INV, LAY, P>(a, grid, st);
        case RO_COLD: return row_one<RO_COLD, LAY, P>(a, grid, st);
        case RO_WARM: return row_one<RO_WARM, LAY, P>(a, grid, st);
        case RO_GS: return row_one<RO_GS, LAY, P>(a, grid, st);
        case RO_GD_FOURIER: return row_one<RO_GD_FOURIER, LAY, P>(a, grid, st);
        case RO_GD_INIT: return row_one<RO_GD_INIT, LAY, P>(a, grid, st);
        case RO_GD: return row_one<RO_GD, LAY, P>(a, grid, st);
        case RO_GS_MID: return row_one<RO_GS_MID, LAY, P>(a, grid, st);
        default: return -1;
    }
}

template <int LAY, int P>
int col_lay(int cw, int op, const mr::ColArgs& a, int grid, hipStream_t st) {
    switch (cw) {
        case 1: return col_cw<1, LAY, P>(op, a, grid, st);
        case 2: return col_cw<2, LAY, P>(op, a, grid, st);
        case 4: return col_cw<4, LAY, P>(op, a, grid, st);
        case 8: return col_cw<8, LAY, P>(op, a, grid, st);
        default: return -1;
    }
}

}  // namespace

// float64: both layouts (panel keys: B2); float32 (the panel shapes' GS): B2 only
int SLM_PASTE(rz_row_launch_, SLM_N)(int prec, int lay, int op, const mr::RowArgs& a, int grid, hipStream_t st) {
    if (prec == PREC_F32) {
        if constexpr (kF32) {
            if (lay == LAY_B2) return row_lay<LAY_B2, PREC_F32>(op, a, grid, st);
        }
        return -1;
    }
    if constexpr (kF64 && kPanel) {
        if (lay == LAY_B2) return row_lay<LAY_B2, PREC_F64>(op, a, grid, st);
    } else if constexpr (kF64) {
        return lay == LAY_B2 ? row_lay<LAY_B2, PREC_F64>(op, a, grid, st) : row_lay<LAY_RM, PREC_F64>(op, a, grid, st);
    }
    return -1;
}

int SLM_PASTE(rz_col_launch_, SLM_N)(int prec, int lay, int cw, int op, const mr::ColArgs& a, int grid, hipStream_t st) {
    if (prec == PREC_F32) {
        if constexpr (kF32) {
            if (lay == LAY_B2) return col_lay<LAY_B2, PREC_F32>(cw, op, a, grid, st);
        }
        return -1;
    }
    if constexpr (kF64 && kPanel) {
        if (lay == LAY_B2) return col_lay<LAY_B2, PREC_F64>(cw, op, a, grid, st);
    } else if constexpr (kF64) {
        return lay == LAY_B2 ? col_lay<LAY_B2, PREC_F64>(cw, op, a, grid, st) : col_lay<LAY_RM, PREC_F64>(cw, op, a, grid, st);
    }
    return -1;
}

int SLM_PASTE(rz_row_rpw_, SLM_N)(int lay) {
    return lay == LAY_B2 ? RowGeo<SLM_N, LAY_B2>::RPW : RowGeo<SLM_N, LAY_RM>::RPW;
}

int SLM_PASTE(rz_col_ok_, SLM_N)(int prec, int cw) {
    if (!(prec == PREC_F32 ? kF32 : kF64)) return 0;
    const bool f32 = prec == PREC_F32;
    switch (cw) {
        case 1: return f32 || kPanel ? 0 : ColGeo<SLM_N, 1>::kValid;
        case 2: return f32 ? ColGeo<SLM_N, 2, PREC_F32>::kValid : ColGeo<SLM_N, 2>::kValid;
        case 4: return f32 ? ColGeo<SLM_N, 4, PREC_F32>::kValid : ColGeo<SLM_N, 4>::kValid;
        case 8: return f32 || kPanel ? 0 : ColGeo<SLM_N, 8>::kValid;
        default: return 0;
    }
}

}  // namespace rz
}  // namespace slm
