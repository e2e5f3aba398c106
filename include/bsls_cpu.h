/*
 * bsls_cpu.h -- C ABI of the host (CPU) path of the c_extensions drop-in.
 *
 * Built from block-simplex-least-squares_amd/cpu/bsls_cpu.cpp into
 * block-simplex-least-squares_amd/lib/libbsls_cpu.so (g++, OpenMP over blocks).
 * Host pointers only.  This is the reference's own CPU c_extensions path
 * (BASELINE configs[0]: main.py BB on the tests/fast problems, no GPU) for
 * callers that select it explicitly (BSLS_DEVICE=cpu, main.py --device cpu);
 * nothing falls back to it: without that selection every entry of the package
 * runs on the MI355X through include/bsls_hip.h and raises without a device.
 *
 * Reference interface each entry replaces (python/c_extensions/):
 *   c_extensions.pyx:22-248 and the header-only kernels it wraps.
 * Same arithmetic order as the reference (bit-identical results); `threads`
 * > 1 spreads independent blocks over OpenMP threads (the result does not
 * depend on it).  Return value: 0, or -1 for invalid arguments.
 */
#ifndef BSLS_CPU_H
#define BSLS_CPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* proj_simplex / proj_multi_simplex / proj_multi_ball (proj_simplex.h:17-74):
 * blocks [starts[b], starts[b+1]) (the last one ends at n), in place. */
int bsls_cpu_proj_simplex(double *y, int64_t start, int64_t end);
int bsls_cpu_proj_multi_simplex(double *y, const int64_t *starts, int64_t nblocks, int64_t n,
                                int threads);
int bsls_cpu_proj_multi_ball(double *y, const int64_t *starts, int64_t nblocks, int64_t n,
                             int threads);

/* isotonic_regression{,_2,_3} and their _multi forms (isotonic_regression.h:
 * 13-164): variant 1, 2 or 3; weight = n int32 run lengths updated in place
 * (unused by variant 2); update = the reference's flag. */
int bsls_cpu_isotonic_multi(int variant, double *y, const int64_t *starts, int64_t nblocks,
                            int64_t n, int32_t *weight, int update, int threads);

/* quad_obj / line_search (quadratic_objective.h:15-61); line_search writes
 * f_new to *f_out (the reference's out-of-bounds store g_new[n] is not made). */
double bsls_cpu_quad_obj(const double *x, const double *Q, const double *c, double *g, int64_t n);
double bsls_cpu_line_search(const double *x, double f, const double *g, double *x_new,
                            double f_new, double *g_new, const double *Q, const double *c,
                            int64_t n);

/* x2z_c / z2x_c (c_extensions.pyx:195-248); starts[0] == 0. */
int bsls_cpu_x2z(const double *x, double *z, const int64_t *starts, int64_t nblocks, int64_t n);
int bsls_cpu_z2x(double *x, const double *z, const int64_t *starts, int64_t nblocks, int64_t n);

const char *bsls_cpu_version(void);

#ifdef __cplusplus
}
#endif
#endif /* BSLS_CPU_H */
