// ref_shim.cpp -- extern "C" entry points over the reference's own header-only
// C++ kernels, compiled from the sources where they lie under /root/reference
// (include path set by oracle/Makefile; nothing is copied into this repo).
//
// TEST INFRASTRUCTURE ONLY: the resulting oracle/_ref/libbsls_ref.so pins the
// oracle restatement (oracle/bsls_oracle.c) and may serve as bench.py's
// "reference" CPU baseline in this container.  It is built only where
// /root/reference exists and is kept out of git history (.gitignore); like every
// other built library it travels in the gpurun snapshot, but no GPU-box process
// loads it (only the CPU pinning tests, tests/test_oracle_pinning.py, do).
//
// Wrapped reference symbols (python/c_extensions/):
//   proj_simplex.h:17,37,50        isotonic_regression.h:13,61,85,95,105,157
//   quadratic_objective.h:15,29
#include "proj_simplex.h"
#include "isotonic_regression.h"
#include "quadratic_objective.h"

extern "C" {

void ref_proj_simplex(double *y, int start, int end) { proj_simplex(y, start, end); }
void ref_proj_multi_simplex(double *y, int *blocks, int nb, int n) {
    proj_multi_simplex(y, blocks, nb, n);
}
void ref_proj_multi_ball(double *y, int *blocks, int nb, int n) {
    proj_multi_ball(y, blocks, nb, n);
}
void ref_isotonic_regression(double *y, int start, int end, int *w, int update) {
    isotonic_regression(y, start, end, w, update);
}
void ref_isotonic_regression_multi(double *y, int *blocks, int nb, int n, int *w,
                                   int update) {
    isotonic_regression_multi(y, blocks, nb, n, w, update);
}
void ref_isotonic_regression_2(double *y, int start, int end) {
    isotonic_regression_2(y, start, end);
}
void ref_isotonic_regression_multi_2(double *y, int *blocks, int nb, int n) {
    isotonic_regression_multi_2(y, blocks, nb, n);
}
void ref_isotonic_regression_3(double *y, int start, int end, int *w, int update) {
    isotonic_regression_3(y, start, end, w, update);
}
void ref_isotonic_regression_multi_3(double *y, int *blocks, int nb, int n, int *w,
                                     int update) {
    isotonic_regression_multi_3(y, blocks, nb, n, w, update);
}
double ref_quad_obj(double *x, double *Q, double *c, double *g, int n) {
    return quad_obj(x, Q, c, g, n);
}
// line_search() stores g_new[n] (one past the end) on its "step too small"
// path; callers must pass g_new with at least n+1 slots.
double ref_line_search(double *x, double f, double *g, double *x_new, double f_new,
                       double *g_new, double *Q, double *c, int n) {
    return line_search(x, f, g, x_new, f_new, g_new, Q, c, n);
}

}  // extern "C"
