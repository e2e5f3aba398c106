/*
 * bsls_hip.h -- C ABI of the MI355X (gfx950) block-simplex least-squares hot path.
 *
 * Built from the .hip sources in block-simplex-least-squares_amd/csrc into
 * block-simplex-least-squares_amd/lib/libbsls_hip.so.  Plain pointers and sizes only:
 * every pointer argument named d_* is DEVICE memory (HBM); `stream` is a
 * hipStream_t passed as void* (NULL = the null stream).  Nothing here takes host
 * buffers: the Python drop-in (c_extensions) stages NumPy inputs itself.
 *
 * Return value: BSLS_OK (0) on success; a positive hipError_t code when a HIP
 * call failed; a negative BSLS_E_* code for invalid arguments.  Launches are
 * asynchronous on `stream`; kernel-side argument faults (e.g. PAVA weights < 1)
 * are reported through the optional d_status word (0 = fine), which the caller
 * reads after synchronising.
 *
 * Reference interface each entry replaces (paths relative to the reference repo):
 *   python/c_extensions/c_extensions.pyx (the Cython module c_extensions) and the
 *   header-only kernels it wraps; SciPy csr_matvec behind A.dot at python/main.py:53-54.
 */
#ifndef BSLS_HIP_H
#define BSLS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BSLS_OK 0
#define BSLS_E_ARG (-1)        /* bad size / null pointer / layout */
#define BSLS_E_WORKSPACE (-2)  /* workspace smaller than *_workspace_size() */
#define BSLS_E_COMM (-100)     /* RCCL missing (exactly this) or failed (minus its ncclResult_t) */

/* Block layout shared by every projection entry: block b covers
 * [d_starts[b], d_starts[b+1]) (the last block ends at n); d_starts strictly
 * increasing, d_starts[0] >= 0, d_starts[nblocks-1] < n; elements before
 * d_starts[0] are left untouched.  max_block = the largest block size (the
 * host knows it; it picks the kernel paths and the workspace size). */

/* ---- simplex / l1-ball projection -------------------------------------------
 * Replaces proj_multi_simplex_c / proj_multi_ball_c (c_extensions.pyx:31-50)
 * -> proj_multi_simplex / proj_multi_ball (proj_simplex.h:37-74).  In place on
 * d_y (fp64).  Bit-identical to the reference for finite inputs. */
size_t bsls_proj_workspace_size(int64_t n, int64_t nblocks, int64_t max_block);
int bsls_proj_multi_simplex(double *d_y, const int64_t *d_starts, int64_t nblocks, int64_t n,
                            int64_t max_block, void *d_work, size_t work_bytes, void *stream);
int bsls_proj_multi_ball(double *d_y, const int64_t *d_starts, int64_t nblocks, int64_t n,
                         int64_t max_block, void *d_work, size_t work_bytes, void *stream);
/* The same two calls (same arguments, workspace and errors) without sorting:
 * lambda from Newton's method on sum_j max(y_j + lambda, 0) = 1 started at the
 * block maximum (the active set only shrinks; the first pass that removes
 * nothing has the reference's set, proj_simplex.h:27-31), the set's sum in a
 * fixed lane order instead of the sorted prefix chain.  Within 1e-12 *
 * max(1, |reference|) of the reference on every tested input (the north
 * star's projection contract), deterministic, not bit-identical. */
int bsls_proj_multi_simplex_fast(double *d_y, const int64_t *d_starts, int64_t nblocks, int64_t n,
                                 int64_t max_block, void *d_work, size_t work_bytes, void *stream);
int bsls_proj_multi_ball_fast(double *d_y, const int64_t *d_starts, int64_t nblocks, int64_t n,
                              int64_t max_block, void *d_work, size_t work_bytes, void *stream);

/* ---- isotonic regression (PAVA) ---------------------------------------------
 * Replaces isotonic_regression_multi_c{,_2,_3} (c_extensions.pyx:76-138) ->
 * isotonic_regression_multi{,_2,_3} (isotonic_regression.h:85-102,157-164).
 * d_weight: run-length array of n int32 (NULL = fresh ones, as weight=None);
 * updated in place like the reference's int weight buffer.  expand = the
 * reference's `update` flag.  Variant 1 is what python/main.py:64 calls.
 * max_block bounds every block length (as for the projections); with
 * variant 1, weight NULL and expand = 1 blocks of <= 64 elements run
 * wave-parallel and longer ones one workgroup each (bit-identical either way). */
size_t bsls_isotonic_workspace_size(int64_t n);
int bsls_isotonic_multi(int variant, double *d_y, const int64_t *d_starts, int64_t nblocks,
                        int64_t n, int32_t *d_weight, int expand, int64_t max_block,
                        void *d_work, size_t work_bytes, int32_t *d_status, void *stream);

/* The same variant-1 call (weight=None, update=1 -- main.py's) on a pack plan
 * made once per block layout: bsls_isotonic_pack_plan (host memory, no GPU)
 * splits the blocks into packs of whole consecutive blocks with <= 64 elements
 * (pk_start: first element, pk_mask: block-start bits relative to it, pk_len:
 * elements) or one longer block (listed in long_packs); call it with
 * pk_start == NULL for the count (returns npacks, *nlong set), then to fill
 * arrays of that size.  bsls_isotonic_packs runs one launch over the device
 * copies (+ one for the long blocks, with the isotonic workspace); the result
 * is bit-identical to bsls_isotonic_multi.  Elements before the first block
 * are untouched. */
int64_t bsls_isotonic_pack_plan(const int64_t *starts, int64_t nblocks, int64_t n,
                                int64_t *pk_start, int64_t *pk_mask, int32_t *pk_len,
                                int32_t *long_packs, int64_t *nlong, int64_t cap);
int bsls_isotonic_packs(double *d_y, const int64_t *d_pk_start, const int64_t *d_pk_mask,
                        const int32_t *d_pk_len, int64_t npacks, const int32_t *d_long_packs,
                        int64_t nlong, int64_t n, void *d_work, size_t work_bytes, void *stream);

/* ---- z <-> x change of variables --------------------------------------------
 * Replaces x2z_c / z2x_c (c_extensions.pyx:195-248); d_starts[0] must be 0. */
int bsls_x2z(const double *d_x, double *d_z, const int64_t *d_starts, int64_t nblocks,
             int64_t n, void *stream);
int bsls_z2x(double *d_x, const double *d_z, const int64_t *d_starts, int64_t nblocks,
             int64_t n, void *stream);

/* N z (with_x0 = 0) or x0 + N z (with_x0 = 1), and g = N' w, for the z-space
 * change of variables (N of bsls_utils.block_sizes_to_N, python/bsls_utils.py:139-162,
 * never materialised): (N z)_i = z_j - z_{j-1} inside a block, last entry -z_last;
 * (N' w)_j = w_i - w_{i+1}.  d_starts are the x-space block starts. */
int bsls_n_apply(double *d_x, const double *d_z, const int64_t *d_starts, int64_t nblocks,
                 int64_t n, int with_x0, void *stream);
int bsls_nt_apply(const double *d_w, double *d_g, const int64_t *d_starts, int64_t nblocks,
                  int64_t n, void *stream);

/* ---- dense QP helpers (not on the sparse hot path; kept for ABI parity) ------
 * Replace quad_obj_c / line_search_quad_obj_c (c_extensions.pyx:148-192) ->
 * quadratic_objective.h:15-61.  The scalar result is written to *d_f (device).
 * line_search: *d_f_out receives f_new; d_x_new / d_g_new updated in place. */
int bsls_quad_obj(const double *d_x, const double *d_Q, const double *d_c, double *d_g,
                  int64_t n, double *d_f, void *stream);
int bsls_line_search(const double *d_x, double f, const double *d_g, double *d_x_new,
                     double f_new, double *d_g_new, const double *d_Q, const double *d_c,
                     int64_t n, double *d_f_out, void *stream);

/* ---- CSR SpMV ----------------------------------------------------------------
 * Replaces scipy csr_matvec behind A.dot(x) (python/main.py:53-54,
 * python/algorithm_utils.py:91-92, python/mirror_descent.py:32-34):
 *   d_out[r] = sum_e data[e] * x[indices[e]]  (+ d_add[r] if d_add)  (* 1 if alpha == 1)
 * int64 row pointers, int32 column indices, fp64 values, one workgroup per
 * host-planned tile (bsls_csr_plan_tiles); `group` = lanes per row in the
 * reduce (power of two 1..64, ~ 256 / rows per tile).  If d_sq_out is
 * non-NULL it receives sum_r d_out[r]^2 (deterministic tree order).
 * The product is alpha * (A x) (alpha == 1.0: no scaling multiply). */
/* Host-side planner (no GPU): split rows [0, m) into tiles of whole rows with
 * <= nzt nonzeros (a single longer row gets its own tile) and <= rmax rows;
 * with `ends` (sorted or not) tiles end only at those row indices.  Writes
 * up to cap+1 row starts into tiles_out (host memory) and returns the tile
 * count (call once with cap = 0 to size), -2 if a forced tile exceeds rmax. */
int64_t bsls_csr_plan_tiles(const int64_t *indptr, int64_t m, int64_t nzt, int64_t rmax,
                            const int64_t *ends, int64_t nends, int64_t *tiles_out, int64_t cap);
size_t bsls_spmv_workspace_size(int64_t ntiles);
int bsls_csr_spmv(int64_t m, const int64_t *d_indptr, const int32_t *d_indices,
                  const double *d_data, const int64_t *d_tiles, int64_t ntiles,
                  const double *d_x, const double *d_add, double alpha, double *d_out,
                  double *d_sq_out, int group, void *d_work, size_t work_bytes, void *stream);

/* ---- fused z-space Barzilai-Borwein engine ----------------------------------
 * Replaces, per iteration, BB.solve's loop body (python/BB.py:17-41) over the
 * closures of main.solve_in_z (python/main.py:53-65) and the stopping rule
 * solvers.stopping (python/solvers.py:40-63):
 *   K1  r = A x + target (= A N z + A x0 - b), ||r||^2, stop test (SpMV, A panels)
 *   K2  g = N' A' r, dg = g - g_prev, BB dot products      (SpMV', explicit A' panels)
 *   K3  z <- clip01(PAVA(z - t g)), x <- N z               (per-block projection)
 * The caller owns every buffer (see struct); bsls_bb_prologue() performs
 * BB.py:14-15 (g_prev = grad(z0 + 1)) and evaluates r(z0).  Iterations keep
 * running until the device-side stop flag is set; after it is set, further
 * enqueued iterations are no-ops.  scal[] layout: BSLS_S_* below. */
enum {
    BSLS_S_STOP = 0,       /* 0 running, else the stop reason BSLS_STOP_* */
    BSLS_S_ITER = 1,       /* last completed iteration i */
    BSLS_S_ZBUF = 2,       /* index (0/1) of the z buffer holding the current iterate */
    BSLS_S_T = 3,          /* last BB step t */
    BSLS_S_FX = 4,         /* f(z) = 0.5 ||r||^2 at the current iterate */
    BSLS_S_SUMDG = 5,      /* sum(delta_g) */
    BSLS_S_DZDG = 6,       /* delta_z . delta_g */
    BSLS_S_DGDG = 7,       /* delta_g . delta_g */
    BSLS_S_GG = 8,         /* g . g */
    BSLS_S_RR = 9,         /* r . r */
    BSLS_S_WARN = 10,      /* count of |t| outside [1e-10, 1e10] (BB.py:27-28) */
    BSLS_S_PSUMDG = 11,    /* stage 10: iteration i - 1's SUMDG, DZDG, DGDG, GG (11..14) */
    BSLS_S_PDZDG = 12, BSLS_S_PDGDG = 13, BSLS_S_PGG = 14,
    BSLS_S_DD = 15,        /* unused (was sy_dr's ||r - r_prev||^2, retired in round 6) */
    BSLS_S_COUNT = 16
};
enum {
    BSLS_STOP_NOCHANGE = 1,   /* BB.py:22  sum(delta_g) == 0 */
    BSLS_STOP_MAXITER = 2,    /* solvers.py:42-44 */
    BSLS_STOP_GRAD = 3,       /* solvers.py:51-54 */
    BSLS_STOP_DG = 4          /* solvers.py:59-62 */
};
/* Panel image of a sparse matrix M (rows x cols) for the fused SpMVs (layout
 * and rationale: csrc/panels.hpp; built on the host by device.build_panels).
 * Rows are cut into panels of `prow` rows (one wave each; K2's panels also
 * carry the next panel's first row, `halo` = 1), 16 panels to a workgroup
 * (row block rb); row r of a panel sits in lane r % 64 of slice r / 64.
 * Columns are cut into chunks that fit the LDS (chunk c = columns
 * [chunk_col[c], chunk_col[c+1]), at most tab_cap wide).  Segment
 * s = (rb * nchunks + c) * 16 + w holds panel 16 rb + w's entries in chunk c:
 * for each slice q with D_q > 0 (D_q = the slice's largest row count in the
 * chunk, bits 16q .. 16q+15 of seg_info[s]), the rows' entries, row after row
 * in column order, each row's run padded to an even length (from ent_off[s],
 * slice after slice), and per row the running total of the padded lengths
 * (inclusive, even) with bit 0 set when the row's own count is odd (cnt,
 * uint16, at cnt_off[s], one group of 64 per such slice; a slice holds
 * < 65535 entries).  An entry is
 * its column offset in the chunk (ent, uint16) and, unless the matrix is a
 * scaled incidence, its value (val). */
#define BSLS_PANEL_CHUNK 20224
#define BSLS_PANEL_ROWS 255
#define BSLS_PANEL_WAVES 16
typedef struct bsls_panels {
    int64_t rows, cols;
    int64_t prow;                   /* rows per panel, 1 .. BSLS_PANEL_ROWS */
    int64_t halo;                   /* 1: panels hold prow + 1 rows (row prow = next panel's row 0) */
    int64_t npanels, nchunks;       /* npanels counts the panels holding rows */
    int64_t ngroups;                /* chunk groups: K1 runs one workgroup per (group, row block) */
    int64_t tab_cap;                /* widest chunk (doubles), 64 .. BSLS_PANEL_CHUNK */
    const int64_t *chunk_col;       /* nchunks + 1 */
    const int64_t *group_chunk;     /* ngroups + 1 */
    const int64_t *ent_off;         /* nsegs + 1: first entry of each segment */
    const int64_t *cnt_off;         /* nsegs + 1: first running count of each segment */
    const int64_t *seg_info;        /* nsegs: D_0 | D_1 << 16 | D_2 << 32 | D_3 << 48 */
    const uint16_t *cnt;
    const uint16_t *ent;            /* + 64 entries of slack at the end */
    const double *val;              /* per entry (+ slack), or NULL when scaled (see colv) */
} bsls_panels;

/* Streamed-tile image of a sparse matrix M (rows x cols): the SpMV format for
 * sparse row blocks, where a panel chunk holds well under one entry per row
 * (config C5: 10M routes over 1M links, ~0.3 entries per row per 20k-column
 * chunk).  Layout and rationale: csrc/tiles.hpp; built on the host by
 * bsls_tiles_build.  Rows are cut into row blocks of H rows (with halo = 1 a
 * block also holds the next block's row 0 as its local row H, for K2's
 * N'w = w_i - w_{i+1}); columns into ngroups groups [group_col[g],
 * group_col[g+1]).  Workgroup (rb, g) of BSLS_TILE_THREADS threads keeps the
 * block's running row sums in LDS; thread t owns the local rows lr with
 * lr % BSLS_TILE_THREADS == t and walks one stream: its rows' entries of group
 * g in column order (every row summed in CSR order, like SciPy's csr_matvec).
 * Wave w of (rb, g) (s = (rb * ngroups + g) * 16 + w) owns the quads (4
 * entries, 16 B) wave_off[s] .. wave_off[s+1] - 1; quad k of its lane l is
 * wave_off[s] + 64 k + l.  Entry = (lr / BSLS_TILE_THREADS) << 24 |
 * (column - group_col[g]) (uint32); a stream shorter than its wave's longest
 * is padded with entries of the dummy slot nslots = ceil((H + halo) / 1024).
 * val: the values in the entries' layout (8 B each), NULL for a scaled
 * incidence.  order: workgroup b -> (rb, g): 0: g = b % ngroups, rb = b /
 * ngroups (with ngroups | 8 every XCD reads one column slice: it stays in the
 * XCD's L2); 1 (ngroups % 8 == 0): XCD x = b % 8 walks its groups x, x + 8, ...
 * one after the other over the launch's row blocks (b / 8 = j * nrb' + rb, g =
 * x + 8 j, nrb' = the row blocks of the launch). */
#define BSLS_TILE_THREADS 1024
#define BSLS_TILE_NT 0x100
/* layouts 1 / 2 with stored values: val holds them as float (VAL32) or
 * _Float16 (VAL16) instead of double -- only when every value converts to that
 * type exactly (checked by the host builder), so the products are the same
 * doubles; 4 or 2 bytes per value instead of 8. */
#define BSLS_TILE_VAL32 0x200
#define BSLS_TILE_VAL16 0x400
#define BSLS_TILE_MAXSLOTS 20       /* LDS: (nslots + 1) * 1024 doubles (x2 with colv) */
/* layout 1 ("dealt"; bsls_tiles_build_dealt): the entries of tile (rb, g) are
 * sorted by column and dealt to the workgroup in that order, so the 64 gathers
 * of one wave-instruction fall in a narrow column range and share cache lines
 * (column-sorted gathers ~2-3x the rate of the thread streams' scattered ones,
 * tools/coal_ubench.hip); the running sums are then added with LDS atomics
 * (ds_add_f64): same sums to rounding, not a fixed order.  Instruction k of a
 * tile (k = (4 s + j) * 16 + w: quad-step s, slot j, wave w) holds up to 64
 * entries whose columns lie in [base_k, base_k + 65535]; entry = local row << 16
 * | (column - group_col[g] - base_k); unused lanes point at the dummy row
 * H + halo.  Tile t = rb * ngroups + g owns quad-steps wave_off[t] ..
 * wave_off[t+1] - 1 (wave_off: nrb * ngroups + 1 entries); quad-step q, wave
 * w, lane l: uint4 ent[(q * 16 + w) * 64 + l] = its slots j = 0..3, bases
 * base[(q * 16 + w) * 4 + j], values val[4 * ((q * 16 + w) * 64 + l) + j].
 * LDS: H + halo + 1 doubles (x2 with colv).  nquads = quad-steps * 1024. */
typedef struct bsls_tiles {
    int64_t rows, cols;
    int64_t H, halo;                /* rows per block; 1: + the next block's row 0 */
    int64_t nrb, ngroups, order;
    int64_t nquads;                 /* ent holds 4 * nquads entries */
    const int64_t *group_col;       /* ngroups + 1 */
    const int64_t *wave_off;        /* layout 0: nrb * ngroups * 16 + 1 (in quads); 1: see above */
    const uint32_t *ent;
    const double *val;              /* 4 * nquads, or NULL (scaled incidence) */
    int64_t layout;                 /* 0: thread streams (CSR order per row), 1: dealt,
                                       2: dealt with 3-byte entries;
                                       | BSLS_TILE_NT: dealt, entries by non-temporal loads;
                                       | BSLS_TILE_VAL32 / VAL16: dealt, narrow exact values */
    const int32_t *base;            /* layout 1: 4 * nquads / 64 instruction bases */
} bsls_tiles;

/* Host-side builder (no device memory): the tile image of the CSR matrix
 * (indptr: rows + 1 int64, indices int32 column-sorted within each row, data
 * optional).  Call once with wave_off_out == NULL to get the quad count
 * (>= 0, or BSLS_E_ARG), allocate 4 * count entries (and values), call again
 * to fill wave_off_out (nrb * ngroups * 16 + 1), ent_out and val_out (when
 * data != NULL).  group_col: ngroups + 1 column bounds. */
int64_t bsls_tiles_build(int64_t rows, int64_t cols, const int64_t *indptr,
                         const int32_t *indices, const double *data, int64_t H, int64_t halo,
                         int64_t ngroups, const int64_t *group_col, int64_t *wave_off_out,
                         uint32_t *ent_out, double *val_out, int64_t nquads_cap);
/* The same for layout 1: call with wave_off_out == NULL for the quad count
 * (quad-steps * 1024), then to fill wave_off_out (nrb * ngroups + 1),
 * ent_out (4 * count), base_out (4 * count / 64) and val_out. */
int64_t bsls_tiles_build_dealt(int64_t rows, int64_t cols, const int64_t *indptr,
                               const int32_t *indices, const double *data, int64_t H,
                               int64_t halo, int64_t ngroups, const int64_t *group_col,
                               int64_t *wave_off_out, uint32_t *ent_out, int32_t *base_out,
                               double *val_out, int64_t nquads_cap);
/* Layout 2: layout 1 with 3-byte entries (local row << cbits | column - base,
 * cbits = 24 - bit_width(H + halo), instructions split where their columns
 * would span more than 2^cbits - 1); lane l of quad-step q, wave w holds its
 * four entries in ent[3 ((q * 16 + w) * 64 + l) + 0..2] as e0 | e1 << 24,
 * e1 >> 8 | e2 << 16, e2 >> 16 | e3 << 8 (ent_out: 3 * count uint32). */
int64_t bsls_tiles_build_dealt3(int64_t rows, int64_t cols, const int64_t *indptr,
                                const int32_t *indices, const double *data, int64_t H,
                                int64_t halo, int64_t ngroups, const int64_t *group_col,
                                int64_t *wave_off_out, uint32_t *ent_out, int32_t *base_out,
                                double *val_out, int64_t nquads_cap);

typedef struct bsls_bb_problem {
    int64_t m, n, nz, nblocks;      /* rows, x length, z length (n - nblocks), blocks */
    bsls_panels A;                  /* K1: A, chunks grouped per XCD (ngroups partials) */
    bsls_panels AT;                 /* K2: A', halo = 1, one group */
    /* scaled incidence (bsls_utils.assert_scaled_incidence, bsls_utils.py:494):
     * every stored entry of column j equals colv[j]; then A.val / AT.val are NULL,
     * x holds colv * (N z) and K2 multiplies by colv of its row.  NULL otherwise. */
    const double *colv;
    double *rpart;                  /* A.ngroups x m partial residuals */
    const double *target;           /* m: A x0 - b (python/main.py:48) */
    const int64_t *xstarts;         /* nblocks, x-space block starts, xstarts[0] = 0 */
    const int64_t *zstarts;         /* nblocks, z-space block starts (xstarts[b] - b) */
    const int32_t *xz;              /* n: z index of x entry i, or -1 for a block's last entry */
    /* K3 packs: runs of whole z-blocks with <= 64 z entries (one wave each), or
     * one block with more (pk_len > 64, serial fallback) */
    const int64_t *pk_z0;           /* first z entry */
    const int64_t *pk_b0;           /* first block */
    const int64_t *pk_mask;         /* block-start bits relative to pk_z0 (uint64) */
    const int32_t *pk_len;          /* z entries */
    int64_t npacks;
    double *z[2];                   /* ping-pong iterate buffers, nz each */
    double *g[2];                   /* ping-pong gradient buffers, nz each */
    double *x;                      /* n: N z of the current iterate (x0 is in target), times colv if set */
    double *r;                      /* m: residual */
    double *scal;                   /* BSLS_S_COUNT doubles */
    void *work;                     /* bsls_bb_workspace_size() bytes; holds dz = z - z_prev
                                     * between iterations, so z[] must not be
                                     * changed between prologue and iterate calls */
    int64_t max_zblock;             /* largest z-block (x-block size - 1) */
    int64_t max_iter;               /* options['max_iter'] */
    double opt_tol;                 /* options['opt_tol'] */
    int32_t early_exit;             /* 0 disables every early exit (fixed-count timing) */
    int32_t shard_role;             /* 0: the whole problem on one GCD; column-sharded
                                     * (bsls_bb_stage 1 is this rank's partial residual):
                                     * 1 = the rank that adds target to its partial, 2 = the
                                     * others, whose stage 1 writes r = 0 once the run has
                                     * stopped (so the all-reduce leaves the final r as it was) */
    /* Tile images replacing the panels when their ent is not NULL (then A / AT
     * are not read): At for K1 (halo 0; ngroups partials in rpart), ATt for K2
     * (halo 1; with ngroups > 1 the partial row sums go through wpart,
     * ngroups * nrb * (H + 1) doubles, then ngroups * nrb slots for stage 8's
     * r^2 slices: ngroups * nrb * (H + 2) doubles in all). */
    bsls_tiles At;
    bsls_tiles ATt;
    double *wpart;
    size_t work_bytes;              /* size of work; < bsls_bb_workspace_size -> BSLS_E_WORKSPACE */
    /* K3's packs of one z-block longer than a wave (pk_len > 64): with
     * long_packs set, K3 leaves them to a follow-up launch of one workgroup per
     * block (PAVA v1 with the whole workgroup, csrc/pava_long.hpp); long_off
     * (nlong + 1) = prefix of their z lengths, long_scratch =
     * bsls_bb_long_scratch_size(long_off[nlong]) bytes.  NULL / 0: K3 runs
     * them serially in one lane. */
    const int32_t *long_packs;
    int64_t nlong;
    const int64_t *long_off;
    void *long_scratch;
    /* colv in a narrower type when every scale converts to it exactly (the
     * host checks; the kernels widen back to the same doubles): colv_codec 1 =
     * float, 2 = _Float16 at colv_n; 0 = read colv itself.  K2's epilogue and K3
     * read the scales of every route per iteration (C5: 80 MB as doubles). */
    const void *colv_n;
    int64_t colv_codec;
    /* Column-sharded sliced schedule (stage 10): the rows [rr_lo, rr_hi) of r
     * whose ||r||^2 this rank sums (1/world of m each; 0, 0: all of them). */
    int64_t rr_lo, rr_hi;
    /* 1: K3 first tests each pack's run partition from its previous call (the
     * fit's partition rarely changes between iterations) and skips the PAVA
     * passes where it still holds (where it fails, its runs that cannot be
     * split stay pooled and the passes continue from them) -- results within
     * ulps of the reference PAVA (the north star's 1e-12), not bit-identical;
     * 0: the reference passes always (bit-identical). */
    int64_t pava_warm;
    /* K1's column-group sums (tile images with several groups): 0 = auto --
     * global f64 atomics into r on a column shard (shard_role 1 / 2), the
     * ordered group partials on one GCD; 1 = always the partials; 2 = atomics
     * wherever K1 has several groups.  (BSLS_K1_ATOMIC=0 / 1 of the Python
     * engine map to 1 / 2, read once when the problem is built.) */
    int64_t k1_atomic;
    /* K3's pack form: 0 = auto (two packs per wave sharing their later PAVA
     * passes from 64k packs on), 1 = one pack per wave, 2 = always two
     * (BSLS_K3_MERGE=0 / 1 of the Python engine). */
    int64_t k3_merge;
    /* > 0: a column shard's r in 64-bit fixed point -- r holds the int64
     * llrint(r_true * r_fx) (r_fx a power of two), so the atomic K1's group
     * sums add as integers (order-free: the same bits whatever order the
     * groups land in) and the all-reduce of r sums int64 (exact: the same bits
     * on every rank count).  Needs the atomic K1 with its initialisation
     * folded into K3 (a dealt K1 image of several groups on shard_role 1 / 2)
     * and a dealt K2 image; every |partial sum| must stay below 2^62 / r_fx
     * (distributed.ShardedBB sizes it from the rows' abs-sums).  0: doubles. */
    double r_fx;
    /* reserved, must be 0 (BSLS_E_ARG otherwise).  Round 5's opt-in delta_z .
     * delta_g as ||r - r_prev||^2 (equal in exact arithmetic) moved where the
     * reference's exact-zero sum(delta_g) exit fires (BB.py:22) and was
     * retired in round 6; K2 sums dz . dg from K3's dz, the reference's
     * expression. */
    int64_t sy_dr;
} bsls_bb_problem;

size_t bsls_bb_workspace_size(int64_t m, int64_t n, int64_t nz);
/* Byte offset in `work` of dz = z - z_prev (nz doubles), the hand-off K3 writes
 * for the next K2 (and the prologue for iteration 1); for tests and tools. */
size_t bsls_bb_dz_offset(int64_t m, int64_t n, int64_t nz);
/* Scratch bytes for K3's long blocks of `total` z entries in all. */
size_t bsls_bb_long_scratch_size(int64_t total);
/* BB.py:14-15 and the first f(z0): resets scal/tickets, g[0] = grad(z0 + 1),
 * r = r(z0), scal[FX] = f(z0).  z[0] must hold z0. */
int bsls_bb_prologue(const bsls_bb_problem *p, void *stream);
/* Enqueue iterations first_iter .. first_iter+count-1 (first_iter >= 1); after
 * iteration i the iterate is z[i & 1] unless the run stopped (scal[ZBUF]). */
int bsls_bb_iterate(const bsls_bb_problem *p, int64_t first_iter, int64_t count, void *stream);
/* The building blocks, for multi-GPU column sharding where RCCL all-reduces sit
 * between them (A_g = the rank's block-aligned column slice):
 *   0  reset scal[] and the reduction tickets
 *   1  r = A_g x_g            (partial residual; all-reduce r afterwards); with
 *      shard_role 1 r = A_g x_g + target (the sum over ranks is the residual)
 *   2  r += target, ||r||^2, f, stopping test of iteration `iter` (iter 0: none)
 *   3  g = N'A'r -> g[iter & 1]; iter > 0 also dg and the four BB sums into
 *      scal[SUMDG..GG] (all-reduce those four afterwards)
 *   4  t from the sums, z[iter&1] = clip01(PAVA(z - t g)), x = N z, dz for stage 3
 *   5  z[1] = z[0] + 1, x = N z[1]           (prologue)
 *   6  x = N z[0]                             (prologue)
 *   7  single GCD: r = A x + target, ||r||^2, f, stopping test (= 1 then 2 fused)
 *   8  stage 3 (iter >= 1) with stage 9 of iteration iter - 1 folded into it:
 *      every workgroup also sums its slice of r^2, and the last one records f
 *      and runs the stopping test of iter - 1 (with the all-reduced g.g of
 *      iter - 1) before it stores iteration iter's four sums
 *   9  ||r||^2, f, stopping test of iteration `iter` (r already the residual)
 *  10  stage 3 (iter >= 1) with this rank's share of ||r||^2 (rows [rr_lo,
 *      rr_hi)) into scal[RR] beside the four sums, iteration iter - 1's sums
 *      kept in scal[PSUMDG..PGG]; all-reduce scal[SUMDG..RR] (5) afterwards
 *  12  f and the stopping test of iteration iter - 1 from those (after the
 *      all-reduce, before stage 4)
 *  13  stage 12 folded into stage 4 (K3's workgroups all decide the stop of
 *      iter - 1 from the same scal values, workgroup 0 records it)
 *  15  stage 13 that also sets r to target (shard_role 1) / 0 for stage 14
 *      when K1 adds its column groups' sums by atomics (a column shard's
 *      dealt K1 with several groups); otherwise stage 13
 *  14  stage 1 after stage 15 (without its own r initialisation then)
 * One iteration i >= 1 = 3, [allreduce sums], 4, 1, [allreduce r], 2; on one GCD
 * bsls_bb_iterate runs 3, 4, 7.  The column-sharded driver (distributed.py,
 * shard_role 1 / 2) runs 8, [allreduce sums], 4, 1, [allreduce r] per
 * iteration and 9 after the last one (fuse 1), or the sliced form 10,
 * [allreduce 5 sums], 15, 14, [allreduce r] (fuse 2, the default; both the
 * native driver bsls_bb_shard_iterate and the Python loop; 13 and 1 where K1
 * runs in row parts, bsls_bb_residual_rows).  After a stop, stage 3 / 8 / 10
 * on a shard_role 2 rank zero its scal[SUMDG..RR], so the all-reduces the
 * driver still enqueues keep the stop iteration's sums (role 1's copy). */
int bsls_bb_stage(const bsls_bb_problem *p, int stage, int64_t iter, void *stream);
/* Stage 1 restricted to K1's row blocks [rb0, rb1) (rows rb0 * R .. rb1 * R - 1,
 * R = *rows_per_block from bsls_bb_row_blocks, which returns the block count):
 * a multi-GPU driver all-reduces r part by part while the next part computes. */
int64_t bsls_bb_row_blocks(const bsls_bb_problem *p, int64_t *rows_per_block);
int bsls_bb_residual_rows(const bsls_bb_problem *p, int64_t iter, int64_t rb0, int64_t rb1,
                          void *stream);

/* ---- LBFGS.solve's weak Wolfe line search on the device ----------------------
 * Replaces weak_wolfe_ls (python/LBFGS.py:9-53) over main.solve_in_z's
 * closures: trial t from 1 by the reference's bisection/doubling, each trial
 * pt = proj(x + t d) (K3: PAVA v1 + clip), f(pt) (K1), the Armijo test
 * f(pt) >= fx + c1 t d.gx, and when it holds g(pt) (K2) and the curvature
 * test d.g(pt) < c2 d.gx; exits as the reference (both hold; |alpha - beta|
 * <= 1e-14; ||t d|| <= 1e-8, taken as |t| ||d||).  Every launch of a trial is
 * gated by the state, so trials enqueued past the exit are no-ops: the host
 * enqueues a few, reads st[] once, enqueues more if needed.  On the accepted
 * exit pt / gpt / S1[FX] are x_next, nabla_f(x_next), f(x_next); after the
 * other two st[T] was never evaluated.  Uses the engine problem's x, r, g and
 * workspace as scratch (its BB state is not kept). */
enum {
    BSLS_LS_T = 0, BSLS_LS_LO = 1, BSLS_LS_HI = 2,  /* t, alpha, beta */
    BSLS_LS_STOP = 3,      /* 0 searching, else BSLS_LS_ACCEPTED / BRACKET / SMALL */
    BSLS_LS_SLOPE = 4,     /* d . gx */
    BSLS_LS_FX = 5,        /* f(x) */
    BSLS_LS_DNORM = 6,     /* ||d|| */
    BSLS_LS_NTRIAL = 7,    /* trials evaluated */
    BSLS_LS_TLAST = 8, BSLS_LS_FT = 9, BSLS_LS_DGT = 10,   /* last trial: t, f(pt), d.g(pt) */
    BSLS_LS_YS = 11, BSLS_LS_GG = 12,   /* after bsls_lbfgs_ls_finish: y.s, g(pt).g(pt) */
    BSLS_LS_DONE = 13,     /* 1 once bsls_lbfgs_ls_finish has run on the accepted trial */
    BSLS_LS_COUNT = 16
};
enum { BSLS_LS_ACCEPTED = 1, BSLS_LS_BRACKET = 2, BSLS_LS_SMALL = 3 };
typedef struct {
    const double *x, *d, *gx;   /* nz each: point (projected), direction, nabla_f(x) */
    double *pt, *gpt;           /* nz each: the trial point and its gradient */
    const double *zero;         /* nz zeros */
    const double *fx;           /* f(x), one device double (may be the last search's
                                   st[BSLS_LS_FT]: begin reads it before resetting st) */
    double *st;                 /* BSLS_LS_COUNT doubles */
    double *S1, *S2;            /* BSLS_S_COUNT doubles each */
    double *part;               /* bsls_lbfgs_ls_work_size(nz) bytes */
    unsigned *tickets;          /* bsls_ticket_bytes() zeroed bytes */
    double c1, c2;              /* 1e-3, 0.9 in the reference */
} bsls_ls_state;
size_t bsls_lbfgs_ls_work_size(int64_t nz);
int bsls_lbfgs_ls_begin(const bsls_bb_problem *p, const bsls_ls_state *s, void *stream);
int bsls_lbfgs_ls_trials(const bsls_bb_problem *p, const bsls_ls_state *s, int64_t count,
                         void *stream);
/* What LBFGS.solve forms after an accepted search (LBFGS.py:100-106): y = g(pt)
 * - gx and s = t d (into y_out / s_out, nz doubles each, when not NULL, with
 * the reference's elementwise roundings), st[YS] = y.s and st[GG] = g(pt).g(pt)
 * (fixed-order block sums), so one read of st[] after the search carries
 * everything the iteration's stopping rule needs.  Gated like the trials:
 * enqueue it after every chunk; it runs once, on the accepted exit only.
 * st[FT] then holds f(pt), and may be passed as the next search's fx. */
int bsls_lbfgs_ls_finish(const bsls_bb_problem *p, const bsls_ls_state *s, double *y_out,
                         double *s_out, void *stream);

/* ---- multi-GPU: one rank's column-sharded iterations, RCCL in the loop ----
 * The reference has no parallel code; this is the driver of
 * distributed.ShardedBB (python) moved to C++ so no Python runs per
 * iteration.  A communicator of `world` ranks (one per GPU, created on the
 * current device; RCCL is resolved at run time from librccl.so.1, so in a
 * torch process it is the RCCL torch.distributed uses): rank 0 makes the id,
 * every rank passes the same bytes to bsls_comm_create. */
typedef struct bsls_comm bsls_comm;
size_t bsls_comm_id_bytes(void);
int bsls_comm_unique_id(void *id_out);
int bsls_comm_create(const void *id, int world, int rank, bsls_comm **out);
int bsls_comm_destroy(bsls_comm *comm);
/* The ranks the communicator spans: RCCL's ncclCommCount for an RCCL
 * communicator, the world it was created with for a callback / model one
 * (bench.py's N > 1 self-check prints it as rccl_ranks). */
int bsls_comm_count(const bsls_comm *comm, int *count_out);
/* A communicator whose all-reduce is a host callback instead of RCCL (a
 * different transport -- MPI, gloo, a test double -- under the same C++
 * driver loop).  fn(d_buf, count, stream, user) must leave the sum over the
 * ranks in d_buf (device memory) ordered after the work already enqueued on
 * `stream` and before the work enqueued after the call returns (e.g.
 * synchronise the stream, reduce, copy back); it returns 0 or nonzero on
 * failure (-> BSLS_E_COMM).  Called on the enqueueing thread, in order.
 * Under a fixed-point r (bsls_bb_problem.r_fx > 0) the r exchange passes
 * r's words, which are int64: the callback must sum them as int64 (the 5-slot
 * scal exchange stays double) -- distributed.CallbackComm does, through the
 * engine's r_exchange view.  bsls_comm_destroy frees it (no RCCL involved). */
typedef int (*bsls_all_reduce_fn)(double *d_buf, int64_t count, void *stream, void *user);
int bsls_comm_create_callback(int world, int rank, bsls_all_reduce_fn fn, void *user,
                              bsls_comm **out);
/* on = 1: bsls_bb_shard_iterate[_parts] run their collectives at world 1 as
 * well (a one-rank sum is the identity, so the results do not change; every
 * RCCL call of the loop -- the five-sum, the r exchange, int64 under a
 * fixed-point r, the parts' exchanges on comm_stream -- then executes on a
 * one-GPU box).  0 (the default): a one-rank communicator skips them. */
int bsls_comm_force_collectives(bsls_comm *comm, int on);
/* in-place sum of `count` doubles over the ranks, on `stream` */
int bsls_comm_all_reduce(bsls_comm *comm, double *d_buf, int64_t count, void *stream);
/* Iterations first_iter .. first_iter+count-1 of the sharded schedule (fuse 2:
 * per iteration stage 10, all-reduce scal[SUMDG..RR], stage 15, stage 14,
 * all-reduce r; fuse 1: stage 8, all-reduce scal[SUMDG..GG], 4, 1,
 * all-reduce r; fuse 0: stage 3 instead of 8 and a stage 9 after every r
 * exchange; stage 9 after the last iteration in all three).  p->shard_role
 * must be 1 on rank 0 and 2 elsewhere (target added once).  A one-rank
 * communicator skips the collectives (a sum over one rank) unless
 * bsls_comm_force_collectives turned them on.  All on
 * `stream`; nothing waits on the host. */
int bsls_bb_shard_iterate(const bsls_bb_problem *p, bsls_comm *comm, int64_t first_iter,
                          int64_t count, int fuse, void *stream);

/* ---- the exchange pipelined behind the walks (link parts) -------------------
 * The K2 image holds `nparts` column groups whose link ranges
 * [group_col[q], group_col[q+1]) are K1's row-block ranges [rb[q] R,
 * rb[q+1] R) (R = the rows per K1 row block, bsls_bb_row_blocks; the last
 * clipped to m).  Then per iteration: K2 part 0 .. nparts-1 (bsls_bb_k2_part:
 * stage 10 on column group q only -- parts < nparts - 1 leave their partial
 * route sums in wpart, the last adds them, runs N' and the sums; part q reads
 * only its rows of r), the five-sum all-reduce, stage 15, and K1 by the same
 * row-block parts (bsls_bb_k1_rows: stage 14 on row blocks [rb0, rb1)), each
 * part's rows of r all-reduced as soon as the part is done -- so part q's
 * exchange runs under K1's later parts and the next K2's earlier parts.
 * bsls_bb_shard_iterate_parts enqueues that (the exchanges on comm_stream,
 * ordered by events; rb_bounds: nparts + 1 host values from 0 to the K1 row
 * block count).  Parts must be launched in order on one stream.
 * bsls_bb_shard_iterate_parts returns BSLS_E_ARG unless the K2 image's
 * group_col[q] == min(rb_bounds[q] R, m) for every q (read from the device
 * once per image and bounds): a part whose columns reached past its exchange
 * would race the all-reduce on comm_stream. */
int bsls_bb_k2_part(const bsls_bb_problem *p, int64_t iter, int part, void *stream);
int bsls_bb_k1_rows(const bsls_bb_problem *p, int64_t iter, int64_t rb0, int64_t rb1,
                    void *stream);
int bsls_bb_shard_iterate_parts(const bsls_bb_problem *p, bsls_comm *comm, int64_t first_iter,
                                int64_t count, int nparts, const int64_t *rb_bounds,
                                void *comm_stream, void *stream);
/* A modelled exchange for one-GPU rehearsals of a rank's share: every
 * "all-reduce" moves nothing and holds its stream for fixed_us + us_per_mb
 * per MB of the buffer (one wave sleeping), so the timing shows how much of
 * an exchange of that cost the schedule hides.  Results are one rank's
 * partial sums: timing only. */
int bsls_comm_create_model(int world, int rank, double fixed_us, double us_per_mb,
                           bsls_comm **out);

/* ---- DORE on the fused images (python/DORE.py:6-90, gradient_descent.py:55-67)
 * The reference loop with linop = scale * A N, linop_T = scale * N'A',
 * proj = PAVA v1 + clip, every branch decided on the device: per iteration i
 *   Ax = linop(x), err = b - Ax, norm_change = ||x - x_prev||^2 (break if i > 0
 *   and <= eps); x_new = proj(x + linop_T(err)) (K2, then K3 with t = -scale);
 *   Ax = linop(x_new), err; i > 2: the two residual extrapolations (a1, a2),
 *   x_2 = proj(x_1 + a2 (x_1 - x_prev)) (K3 with t = -a2), Ax_2, and x_2 kept
 *   when ||err_2||^2 / ||err||^2 < 1.
 * Buffers rotate by iteration: x = X[i%3], x_prev = X[(i+2)%3], the new x is
 * written to X[(i+1)%3]; AX[i%3] = Ax at the end of iteration i.  S / S2 are
 * scal[] blocks (BSLS_S_*) gating the main and the extrapolated path (S:
 * SUMDG = 1, DZDG = -scale, DGDG = 1, STOP = 0 before the first call);
 * dsc[BSLS_DORE_*] the loop's scalars.  K1 / K2 / K3 use p's images and work. */
enum {
    BSLS_DORE_NC = 0,      /* norm_change of the last iteration */
    BSLS_DORE_EE = 1,      /* err.err after linop(x_new) */
    BSLS_DORE_A1 = 2,
    BSLS_DORE_A2 = 3,
    BSLS_DORE_SEL = 4,     /* 1: x_2 selected in the last iteration */
    BSLS_DORE_STOPIT = 5,  /* iteration of the norm-change break (S[STOP] = 1) */
    BSLS_DORE_COUNT = 16
};
typedef struct bsls_dore_state {
    double *X[3];          /* nz each */
    double *X1, *D, *X2;   /* x_1, x_1 - x_prev, x_2: nz each */
    double *AX[3];         /* m each */
    double *AX2, *err, *b; /* m each; b = -scale * target (DORE.py:23) */
    double *S, *S2;        /* BSLS_S_COUNT doubles each */
    double *dsc;           /* BSLS_DORE_COUNT doubles */
    double *part;          /* bsls_dore_work_size(nz, m) bytes: reduction partials */
    unsigned *tickets;     /* bsls_ticket_bytes() zeroed bytes (nine 64-B ticket words) */
    double scale, eps;
} bsls_dore_state;
size_t bsls_dore_work_size(int64_t nz, int64_t m);
/* Bytes of one set of reduction tickets (bsls_dore_state.tickets). */
size_t bsls_ticket_bytes(void);
int bsls_dore_iterate(const bsls_bb_problem *p, const bsls_dore_state *d, int64_t first_iter,
                      int64_t count, void *stream);

/* ---- x-space least-squares operator on panel images -------------------------
 * Replaces sparse_least_squares_obj's two SciPy products
 * (python/algorithm_utils.py:88-94; python/mirror_descent.py:31-34):
 *   bsls_lsq_residual   r = A x + add (add may be NULL), *sq_out = ||r||^2
 *                       (device double, optional; fixed-order reduction)
 *   bsls_lsq_gradient   g = A' r  (rows of A' summed in CSR order: bit-identical
 *                       to SciPy's csr_matvec)
 * A: panels with its columns in ngroups groups, halo 0 (as bsls_bb_problem.A);
 * AT: A' panels, halo 0, one group.  Scaled incidence (colv != NULL): values
 * not stored, xs (n doubles) is scratch for colv * x. */
typedef struct bsls_lsq_op {
    int64_t m, n;
    bsls_panels A;
    bsls_panels AT;
    const double *colv;             /* n, or NULL (A.val / AT.val stored) */
    double *rpart;                  /* A.ngroups x m partial residuals */
    double *xs;                     /* n scratch (scaled only) */
    void *work;                     /* bsls_lsq_workspace_size() bytes, zeroed once */
    size_t work_bytes;
    /* Optional dealt tile image of A (layout 1 / 2, halo 0): when At.ent is set
     * the residual walks it instead of the A panels (LDS atomic row sums, the
     * z-space K1's walk; rpart then holds At.ngroups x m) and op->A is unused. */
    bsls_tiles At;
    /* Optional dealt tile image of A' (layout 1 / 2, one group, halo 0): when
     * ATt.ent is set the gradient walks it instead of the AT panels (LDS
     * atomic row sums scaled by colv once per row: g to rounding, not SciPy's
     * order; mirror descent) and op->AT is unused. */
    bsls_tiles ATt;
    /* 1 (with At, dealt): the residual's row sums in 64-bit fixed point,
     * order-free -- r and ||r||^2 repeat bit for bit at the same x, at the
     * dealt walk's speed (the x-space solvers' exits compare f across rounds).
     * fx_amax >= max_i sum_j |A_ij| (a scaled incidence: the most entries in a
     * row); the scale is set per call from fx_amax * max|x|, each term rounds
     * to 2^-50 of that bound. */
    int64_t fixed;
    double fx_amax;
    /* fixed only: > 0 is the caller's guarantee that max|x| (of colv * x with a
     * scaled incidence) <= x_bound for this call, so the per-call max pass is
     * skipped (an x-space solver's projected iterates: |x| <= 1 per entry);
     * 0 = the max is measured per call.  A violated bound corrupts r. */
    double x_bound;
} bsls_lsq_op;

size_t bsls_lsq_workspace_size(int64_t m, int64_t A_npanels);
int bsls_lsq_residual(const bsls_lsq_op *op, const double *d_x, const double *d_add, double *d_r,
                      double *d_sq_out, void *stream);
int bsls_lsq_gradient(const bsls_lsq_op *op, const double *d_r, double *d_g, void *stream);

/* ---- fused x-space Barzilai-Borwein engine ----------------------------------
 * Replaces BATCH.solve_BB (python/BATCH.py:55-106) over the closures of
 * algorithm_utils.get_solver_parts(is_sparse=True) (python/algorithm_utils.py:
 * 182-271): obj = sparse_least_squares_obj (:88-94), proj = proj_multi_simplex
 * / proj_multi_ball, line_search = line_search_np (:113-137), and the stopping
 * rule algorithm_utils.stopping (:158-172).
 * The device runs ROUNDS; a round is either one BB step (x_new = proj(x - t g),
 * obj(x_new), Armijo test) or one backtracking step of the line search
 * (x_new = (1-tt) x + tt x_new, obj(x_new), test) -- which one is decided on
 * the device, so the host only enqueues rounds (5 launches each) and polls
 * scal[XS_MODE] for BSLS_XM_STOPPED.  Rounds after the stop are no-ops.
 * scal[] layout: BSLS_XS_*; hist[k] = f after iteration k (hist[0] = f(x0)),
 * the reference's progress[k][1], for k < hist_cap. */
enum {
    BSLS_XS_MODE = 0,      /* BSLS_XM_* of the next round */
    BSLS_XS_ITER = 1,      /* the reference's i */
    BSLS_XS_F = 2,         /* f at x */
    BSLS_XS_FOLD = 3,      /* f_old */
    BSLS_XS_T = 4,         /* BB step of the next STEP round */
    BSLS_XS_TT = 5,        /* line-search t of the next BACKTRACK round */
    BSLS_XS_REVERT = 6,    /* 1: the next BACKTRACK round restores x (step too small) */
    BSLS_XS_GD = 7,        /* g . (x_new - x) of the last round */
    BSLS_XS_DXDG = 8,      /* delta_x . delta_g of the last accepted step */
    BSLS_XS_DGDG = 9,      /* delta_g . delta_g of the last accepted step */
    BSLS_XS_STEPINF = 10,  /* ||x_new - x||_inf of the last round */
    BSLS_XS_SQ = 11,       /* ||A x_new - b||^2 of the last round */
    BSLS_XS_STOP = 12,     /* BSLS_XSTOP_* (the LAST matching test, like the reference) */
    BSLS_XS_ROUNDS = 13,   /* rounds run */
    BSLS_XS_BACKTRACKS = 14,
    BSLS_XS_COUNT = 16
};
enum { BSLS_XM_INIT = 0, BSLS_XM_STEP = 1, BSLS_XM_BACKTRACK = 2, BSLS_XM_STOPPED = 3 };
enum { BSLS_XSTOP_MAXITER = 1, BSLS_XSTOP_OPT = 2, BSLS_XSTOP_PROG = 3 };

typedef struct bsls_csr {           /* a CSR matrix for bsls_csr_spmv */
    int64_t rows;
    const int64_t *indptr;
    const int32_t *indices;
    const double *data;
    const int64_t *tiles;           /* bsls_csr_plan_tiles */
    int64_t ntiles;
    int64_t group;
} bsls_csr;

typedef struct bsls_xbb_problem {
    int64_t m, n, nblocks, max_block;
    int64_t ball;                   /* bit 0: proj_multi_ball (else proj_multi_simplex);
                                       bit 1: the sort-free _fast form */
    bsls_csr A, AT;                 /* A (m x n) and A' (n x m), explicit */
    const double *neg_b;            /* m: -b */
    const int64_t *starts;          /* nblocks block starts (strictly increasing) */
    double *x, *g, *xn, *gn;        /* n each: iterate, gradient, trial point, its gradient */
    double *r;                      /* m */
    double *scal;                   /* BSLS_XS_COUNT */
    double *hist;                   /* hist_cap */
    int64_t hist_cap;
    void *proj_work;                /* bsls_proj_workspace_size(n, nblocks, max_block) */
    size_t proj_work_bytes;
    void *work;                     /* bsls_xbb_workspace_size() bytes, zeroed once */
    size_t work_bytes;
    int64_t max_iter;
    double opt_tol, prog_tol, f_min;
    int64_t has_fmin;
    const bsls_lsq_op *lsq;         /* panel operator for both products, or NULL (A / AT CSR) */
    /* L-BFGS (BATCH.solve_LBFGS, python/BATCH.py:110-214): lbfgs = corrections
     * C > 0 replaces the BB step of iterations i > 5 by the two-loop recursion
     * of LBFGS_helper (:196-214) over the history queues; i <= 5 keep the BB
     * step (:179-181).  As in the reference, the queues hold the one delta_x /
     * delta_g buffer that every iteration overwrites, so every stored
     * correction is the latest (s, y) with its own rho: the recursion runs in
     * the coefficients of d = a g + b s + c y (four dot products per
     * iteration, one pass; then x_new = x + d, one pass).  0: BB. */
    int64_t lbfgs;
    double *s, *y;                  /* n each: delta_x, delta_g of the last accepted step */
    double *lb;                     /* bsls_xbb_lbfgs_size(lbfgs) BYTES: rho ring, alpha, coefficients */
} bsls_xbb_problem;

size_t bsls_xbb_workspace_size(int64_t m, int64_t n, int64_t A_ntiles, int64_t AT_ntiles);
/* Bytes of the L-BFGS scratch `lb` for `corrections` (0: none). */
size_t bsls_xbb_lbfgs_size(int64_t corrections);
/* x must hold x_init; resets scal (mode INIT) and the reduction tickets. */
int bsls_xbb_init(const bsls_xbb_problem *p, void *stream);
/* Enqueue `count` rounds (the first one after init evaluates obj(x_init)). */
int bsls_xbb_rounds(const bsls_xbb_problem *p, int64_t count, void *stream);

/* ---- mirror descent ---------------------------------------------------------
 * Replaces mirror_descent.least_squares's step (python/mirror_descent.py:37-47):
 * x <- x * exp(-t_k g) per coordinate, t_k = sqrt(2 ln k_b)/(sqrt(k) Lf), then
 * every block divided by its sum; *d_dxinf receives ||x_new - x_old||_inf.
 * d_g = A'(Ax - b) computed with bsls_csr_spmv.  In place on d_x. */
int bsls_md_update(double *d_x, const double *d_g, const int64_t *d_starts, int64_t nblocks,
                   int64_t n, double step_scale, double *d_dxinf, void *d_work,
                   size_t work_bytes, void *stream);
size_t bsls_md_workspace_size(int64_t nblocks);

/* The same update with the reference's stopping test on the device, so the
 * host need not read ||x_new - x_old||_inf every iteration
 * (mirror_descent.py:50-51): d_state[3] = {stopped, last norm, stop
 * iteration}, zeroed by the caller before iteration 1; once the norm of
 * iteration `iter` is < tol, state = {1, norm, iter} and later calls leave x
 * unchanged. */
int bsls_md_update_gated(double *d_x, const double *d_g, const int64_t *d_starts, int64_t nblocks,
                         int64_t n, double step_scale, double tol, int64_t iter, double *d_state,
                         void *d_work, size_t work_bytes, void *stream);

/* The gated update over host-planned packs of whole blocks (one wave each,
 * <= 64 entries one per lane, or one block > 64 entries): pk_x0 first entry,
 * pk_mask block-start bits (bit 0 set), pk_len entries.  Coalesced, one exp
 * per entry; block sums in a fixed tree order (within 1e-15 of the
 * left-to-right sum).  d_state as for bsls_md_update_gated. */
size_t bsls_md_pack_workspace_size(int64_t npacks);
int bsls_md_update_packs(double *d_x, const double *d_g, const int64_t *d_pk_x0,
                         const int64_t *d_pk_mask, const int32_t *d_pk_len, int64_t npacks,
                         double step_scale, double tol, int64_t iter, double *d_state,
                         void *d_work, size_t work_bytes, void *stream);

/* Replaces BATCH.solve_MD's update (python/BATCH.py:238-240) and
 * algorithm_utils.normalization (python/algorithm_utils.py:175-179):
 * d_y = d_x * exp(-t d_g) (d_y = d_x when d_g is NULL), then every block
 * [starts[b], starts[b+1]) (last block to n) divided by its sum.  d_y may
 * alias d_x. */
int bsls_md_step(const double *d_x, const double *d_g, double *d_y, const int64_t *d_starts,
                 int64_t nblocks, int64_t n, double t, void *stream);

/* ---- LBFGS.solve's direction (python/LBFGS.py:59-71), vector-free ----------
 * The two-loop recursion over the m stored pairs runs on dot products: one
 * pass computing every dot an iteration needs, the m-step loops on scalars in
 * one wave, one combine pass.  Replaces the 2m dependent dots and 2m AXPYs of
 * `direction` (python/LBFGS.py:59-71) and the list rotation of :75-77.
 *
 * bsls_multi_dot: d_out[j * K + k] = d_rows[j] . d_cols[k] (1 <= J <= 4;
 * d_rows / d_cols are DEVICE arrays of device pointers, every vector n
 * doubles).  Fixed summation order (deterministic). */
size_t bsls_multi_dot_workspace_size(int64_t J, int64_t K);
int bsls_multi_dot(const double *const *d_rows, int J, const double *const *d_cols, int K,
                   int64_t n, double *d_out, void *d_work, size_t work_bytes, void *stream);
/* d_out[i] = sum_k d_coef[k] * d_vecs[k][i], k ascending (1 <= K <= 256). */
int bsls_multi_axpy(const double *const *d_vecs, int K, const double *d_coef, int64_t n,
                    double *d_out, void *stream);
/* History state of m <= 127 pairs (ring slot (head + k) % m = pair k, 0 the
 * oldest): rho[m], SY[m][m] (s_a . y_b), YY[m][m], coef[2m + 1], scratch;
 * zero-initialised = the reference's m zero pairs (LBFGS.py:51). */
size_t bsls_lbfgs_state_size(int64_t m);
/* d_dots: bsls_multi_dot of rows {g_new, y_new, s_new} against columns
 * {S slot 0..m-1, Y slot 0..m-1, y_new, s_new} (K = 2m + 2).  Writes
 * coef = [a, b_0..b_{m-1}, c_0..c_{m-1}] with d = a g_new + sum b_j S_j +
 * sum c_j Y_j the reference's `direction` (H from y_new, s_new). */
int bsls_lbfgs_coef(int64_t m, int64_t head, double *d_state, const double *d_dots,
                    void *stream);
/* Pushes (y_new, s_new, rho_new) into ring slot `slot` (the oldest, = head):
 * copies the vectors, fills the slot's Gram rows from the same d_dots. */
int bsls_lbfgs_push(int64_t m, int64_t slot, double rho_new, double *d_state,
                    const double *d_dots, const double *d_y_new, const double *d_s_new,
                    double *d_y_slot, double *d_s_slot, int64_t n, void *stream);

/* Library / device info (for the loader's self-check). */
const char *bsls_version(void);
int bsls_device_arch(char *buf, int buflen);

#ifdef __cplusplus
}
#endif
#endif /* BSLS_HIP_H */
