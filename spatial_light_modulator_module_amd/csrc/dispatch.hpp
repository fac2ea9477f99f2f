// Host-side lookup of the per-length kernel instantiations.
#pragma once
#include <hip/hip_runtime.h>

namespace slm {

struct RowParams;
struct ColParams;
using RowFn = void (*)(RowParams);
using ColFn = void (*)(ColParams);

#define SLM_DECLARE_LENGTH(N)                    \
    RowFn row_fn_##N(int mode, int prec);                  \
    ColFn col_fn_##N(int cw, int mode, int tt, int prec);  \
    int row_threads_##N();                       \
    int row_rpw_##N();                           \
    int col_threads_##N(int cw);

SLM_DECLARE_LENGTH(64)
SLM_DECLARE_LENGTH(128)
SLM_DECLARE_LENGTH(256)
SLM_DECLARE_LENGTH(512)
SLM_DECLARE_LENGTH(768)
SLM_DECLARE_LENGTH(1024)
SLM_DECLARE_LENGTH(2048)
SLM_DECLARE_LENGTH(4096)

#define SLM_FOR_EACH_LENGTH(X) X(64) X(128) X(256) X(512) X(768) X(1024) X(2048) X(4096)

inline RowFn row_fn(int n, int mode, int prec) {
#define SLM_CASE(N) \
    case N: return row_fn_##N(mode, prec);
    switch (n) { SLM_FOR_EACH_LENGTH(SLM_CASE) default: return nullptr; }
#undef SLM_CASE
}
inline ColFn col_fn(int n, int cw, int mode, int tt, int prec) {
#define SLM_CASE(N) \
    case N: return col_fn_##N(cw, mode, tt, prec);
    switch (n) { SLM_FOR_EACH_LENGTH(SLM_CASE) default: return nullptr; }
#undef SLM_CASE
}
inline int row_threads(int n) {
#define SLM_CASE(N) \
    case N: return row_threads_##N();
    switch (n) { SLM_FOR_EACH_LENGTH(SLM_CASE) default: return 0; }
#undef SLM_CASE
}
inline int row_rpw(int n) {
#define SLM_CASE(N) \
    case N: return row_rpw_##N();
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
