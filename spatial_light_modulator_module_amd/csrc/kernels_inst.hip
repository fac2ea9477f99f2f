// Instantiates every row / column kernel of one radix plan (plan key SLM_N,
// an index into kPlans). Compiled once per plan (see Makefile) so the builds
// run in parallel; dispatch.hpp maps (plan key, mode, ...) to these tables.
#include "dispatch.hpp"
#include "kernels.hpp"

#ifndef SLM_N
#error "compile with -DSLM_N=<plan key>"
#endif

#define SLM_PASTE2(a, b) a##b
#define SLM_PASTE(a, b) SLM_PASTE2(a, b)

namespace slm {
namespace {

template <int N, int P, int LID>
RowFn row_table(int mode) {
    switch (mode) {
        case ROW_GS_MAIN: return row_kernel<N, ROW_GS_MAIN, P, LID>;
        case ROW_GS_PHASE: return row_kernel<N, ROW_GS_PHASE, P, LID>;
        case ROW_PHASE_FWD: return row_kernel<N, ROW_PHASE_FWD, P, LID>;
        case ROW_GD_INIT_Y: return row_kernel<N, ROW_GD_INIT_Y, P, LID>;
        case ROW_GD_INIT_FIELD: return row_kernel<N, ROW_GD_INIT_FIELD, P, LID>;
        case ROW_GD_MAIN: return row_kernel<N, ROW_GD_MAIN, P, LID>;
        case ROW_FFT_FWD: return row_kernel<N, ROW_FFT_FWD, P, LID>;
        case ROW_FFT_INV: return row_kernel<N, ROW_FFT_INV, P, LID>;
        case ROW_GD_LIN: return row_kernel<N, ROW_GD_LIN, P, LID>;
        default: return nullptr;
    }
}

template <int N, int CW, int P, int LID>
ColFn col_table_cw(int mode, int tt) {
    if constexpr (!ColCfg<N, CW>::kValid) {
        return nullptr;
    } else {
        const bool u8 = (tt == TGT_U8);
        switch (mode) {
            case COL_GS_MAIN:  // GS plans hold a float32 target as its amplitude (TGT_AMP)
                return u8 ? col_kernel<N, CW, COL_GS_MAIN, TGT_U8, P, LID>
                          : tt == TGT_AMP ? col_kernel<N, CW, COL_GS_MAIN, TGT_AMP, P, LID> : nullptr;
            case COL_REAL_INV:
                return u8 ? col_kernel<N, CW, COL_REAL_INV, TGT_U8, P, LID>
                          : tt == TGT_AMP ? col_kernel<N, CW, COL_REAL_INV, TGT_AMP, P, LID>
                                          : col_kernel<N, CW, COL_REAL_INV, TGT_F32, P, LID>;
            case COL_GD_STATS:
                return u8 ? col_kernel<N, CW, COL_GD_STATS, TGT_U8, P, LID> : col_kernel<N, CW, COL_GD_STATS, TGT_F32, P, LID>;
            case COL_GD_GRAD:
                return u8 ? col_kernel<N, CW, COL_GD_GRAD, TGT_U8, P, LID> : col_kernel<N, CW, COL_GD_GRAD, TGT_F32, P, LID>;
            case COL_GD_FUSED:  // float32 GD only (the 1-launch GD column side)
                if constexpr (P == PREC_F32)
                    return u8 ? col_kernel<N, CW, COL_GD_FUSED, TGT_U8, P, LID> : col_kernel<N, CW, COL_GD_FUSED, TGT_F32, P, LID>;
                else
                    return nullptr;
            case COL_GD_LIN:
                return u8 ? col_kernel<N, CW, COL_GD_LIN, TGT_U8, P, LID> : col_kernel<N, CW, COL_GD_LIN, TGT_F32, P, LID>;
            case COL_EXPECTED: return col_kernel<N, CW, COL_EXPECTED, TGT_F32, P, LID>;
            case COL_FFT_FWD: return col_kernel<N, CW, COL_FFT_FWD, TGT_F32, P, LID>;
            case COL_FFT_INV: return col_kernel<N, CW, COL_FFT_INV, TGT_F32, P, LID>;
            default: return nullptr;
        }
    }
}

template <int N, int P, int LID>
ColFn col_table(int cw, int mode, int tt) {
    switch (cw) {
        case 1: return col_table_cw<N, 1, P, LID>(mode, tt);
        case 2: return col_table_cw<N, 2, P, LID>(mode, tt);
        case 4: return col_table_cw<N, 4, P, LID>(mode, tt);
        case 8: return col_table_cw<N, 8, P, LID>(mode, tt);
        case 16: return col_table_cw<N, 16, P, LID>(mode, tt);
        default: return nullptr;
    }
}

template <int LID>
RowFn row_fn_lid(int mode, int prec) {
    return prec == PREC_F64 ? row_table<SLM_N, PREC_F64, LID>(mode) : row_table<SLM_N, PREC_F32, LID>(mode);
}
ColFn col_fn_default(int cw, int mode, int tt, int prec) {
    return prec == PREC_F64 ? col_table<SLM_N, PREC_F64, LAYOUT_DEFAULT>(cw, mode, tt)
                            : col_table<SLM_N, PREC_F32, LAYOUT_DEFAULT>(cw, mode, tt);
}

}  // namespace

// layout pair `lid` (LayoutId); nullptr where this plan is not built with it
RowFn SLM_PASTE(row_fn_, SLM_N)(int mode, int prec, int lid) {
    if (lid == LAYOUT_DEFAULT) return row_fn_lid<LAYOUT_DEFAULT>(mode, prec);
    if constexpr (kHasNarrowLayout<SLM_N>)
        if (lid == LAYOUT_NARROW) return row_fn_lid<LAYOUT_NARROW>(mode, prec);
    return nullptr;
}

ColFn SLM_PASTE(col_fn_, SLM_N)(int cw, int mode, int tt, int prec, int lid) {
    if (lid == LAYOUT_DEFAULT) return col_fn_default(cw, mode, tt, prec);
    if constexpr (kHasNarrowLayout<SLM_N>)  // 2-column tiles only
        if (lid == LAYOUT_NARROW && cw == 2)
            return prec == PREC_F64 ? col_table_cw<SLM_N, 2, PREC_F64, LAYOUT_NARROW>(mode, tt)
                                    : col_table_cw<SLM_N, 2, PREC_F32, LAYOUT_NARROW>(mode, tt);
    return nullptr;
}

int SLM_PASTE(row_threads_, SLM_N)(int prec) {
    return prec == PREC_F64 ? RowCfg<SLM_N, PREC_F64>::THREADS : RowCfg<SLM_N, PREC_F32>::THREADS;
}
int SLM_PASTE(row_rpw_, SLM_N)(int prec) {
    return prec == PREC_F64 ? RowCfg<SLM_N, PREC_F64>::RPW : RowCfg<SLM_N, PREC_F32>::RPW;
}
int SLM_PASTE(col_threads_, SLM_N)(int cw) {
    switch (cw) {
        case 1: return ColCfg<SLM_N, 1>::THREADS;
        case 2: return ColCfg<SLM_N, 2>::THREADS;
        case 4: return ColCfg<SLM_N, 4>::THREADS;
        case 8: return ColCfg<SLM_N, 8>::THREADS;
        case 16: return ColCfg<SLM_N, 16>::THREADS;
        default: return 0;
    }
}

}  // namespace slm
