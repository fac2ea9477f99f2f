// Host-side lookup of the per-plan kernel instantiations (keyed by plan key).
#pragma once
#include <hip/hip_runtime.h>

#include "plans.hpp"

namespace slm {

struct RowParams;
struct ColParams;
using RowFn = void (*)(RowParams);
using ColFn = void (*)(ColParams);

#define SLM_DECLARE_LENGTH(N)                    \
    RowFn row_fn_##N(int mode, int prec, int lid);         \
    ColFn col_fn_##N(int cw, int mode, int tt, int prec, int lid); \
    int row_threads_##N(int prec);               \
    int row_rpw_##N(int prec);                   \
    int col_threads_##N(int cw);

SLM_DECLARE_LENGTH(0)
SLM_DECLARE_LENGTH(1)
SLM_DECLARE_LENGTH(2)
SLM_DECLARE_LENGTH(3)
SLM_DECLARE_LENGTH(4)
SLM_DECLARE_LENGTH(5)
SLM_DECLARE_LENGTH(6)
SLM_DECLARE_LENGTH(7)
SLM_DECLARE_LENGTH(8)
SLM_DECLARE_LENGTH(9)
SLM_DECLARE_LENGTH(10)
SLM_DECLARE_LENGTH(11)
SLM_DECLARE_LENGTH(12)
SLM_DECLARE_LENGTH(13)

// plan keys (indices into kPlans); the Makefile builds one object per key
static_assert(kNumF32Plans == 14, "update SLM_DECLARE_LENGTH / SLM_FOR_EACH_LENGTH and the Makefile");
#define SLM_FOR_EACH_LENGTH(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13)

inline RowFn row_fn(int n, int mode, int prec, int lid = 0) {
#define SLM_CASE(N) \
    case N: return row_fn_##N(mode, prec, lid);
    switch (n) { SLM_FOR_EACH_LENGTH(SLM_CASE) default: return nullptr; }
#undef SLM_CASE
}
inline ColFn col_fn(int n, int cw, int mode, int tt, int prec, int lid = 0) {
#define SLM_CASE(N) \
    case N: return col_fn_##N(cw, mode, tt, prec, lid);
    switch (n) { SLM_FOR_EACH_LENGTH(SLM_CASE) default: return nullptr; }
#undef SLM_CASE
}
inline int row_threads(int n, int prec) {
#define SLM_CASE(N) \
    case N: return row_threads_##N(prec);
    switch (n) { SLM_FOR_EACH_LENGTH(SLM_CASE) default: return 0; }
#undef SLM_CASE
}
inline int row_rpw(int n, int prec) {
#define SLM_CASE(N) \
    case N: return row_rpw_##N(prec);
    switch (n) { SLM_FOR_EACH_LENGTH(SLM_CASE) default: return 0; }
#undef SLM_CASE
}
inline int col_threads(int n, int cw) {
#define SLM_CASE(N) \
    case N: return col_threads_##N(cw);
    switch (n) { SLM_FOR_EACH_LENGTH(SLM_CASE) default: return 0; }
#undef SLM_CASE
}

}  // namespace slm
