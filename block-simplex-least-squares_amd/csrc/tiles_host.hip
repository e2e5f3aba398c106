// tiles_host.hip -- host-side builder of the streamed-tile image
// (include/bsls_hip.h, struct bsls_tiles; device side csrc/tiles.hpp).
//
// Pure host code (no device memory).  Two passes over the CSR rows of each row
// block: count the entries per (group, owning thread) to size every wave's
// stream (its longest lane, in 4-entry quads), then bucket, sort each thread's
// entries by column and scatter them into the interleaved quads.  Row blocks
// are independent: they are spread over host threads (a C5 image, 160M
// entries, builds in a few seconds instead of the minutes NumPy argsorts take).
#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "tiles.hpp"

using namespace bsls;

namespace {

struct Plan {
    int64_t rows, cols, H, halo, nrb, G, nslots;
    const int64_t *indptr;
    const int32_t *indices;
    const int64_t *gc;
    std::vector<int32_t> gmap;   // column -> group
};

// rows of block rb in local order: [rb H, min(rb H + H + halo, rows))
inline int64_t block_end(const Plan &p, int64_t rb) {
    return std::min(p.rows, rb * p.H + p.H + p.halo);
}

template <typename F>
void parallel_blocks(int64_t nrb, F f) {
    unsigned nt = std::thread::hardware_concurrency();
    nt = std::max(1u, std::min(nt, 16u));
    if (nrb < 2 || nt == 1) {
        for (int64_t rb = 0; rb < nrb; ++rb) f(rb);
        return;
    }
    std::atomic<int64_t> next(0);
    std::vector<std::thread> th;
    for (unsigned k = 0; k < nt; ++k)
        th.emplace_back([&]() {
            for (int64_t rb; (rb = next.fetch_add(1)) < nrb;) f(rb);
        });
    for (auto &x : th) x.join();
}

// per-thread entry counts of block rb, (g, t) -> cnt[g * T + t]
void count_block(const Plan &p, int64_t rb, std::vector<int64_t> &cnt) {
    cnt.assign((size_t)p.G * TILE_T, 0);
    const int64_t r0 = rb * p.H;
    for (int64_t i = r0; i < block_end(p, rb); ++i) {
        const int t = (int)((i - r0) % TILE_T);
        for (int64_t k = p.indptr[i]; k < p.indptr[i + 1]; ++k)
            cnt[(size_t)p.gmap[p.indices[k]] * TILE_T + t]++;
    }
}

}  // namespace

extern "C" int64_t bsls_tiles_build(int64_t rows, int64_t cols, const int64_t *indptr,
                                    const int32_t *indices, const double *data, int64_t H,
                                    int64_t halo, int64_t ngroups, const int64_t *group_col,
                                    int64_t *wave_off_out, uint32_t *ent_out, double *val_out,
                                    int64_t nquads_cap) {
    if (rows < 1 || cols < 1 || !indptr || !indices || H < 64 || (halo != 0 && halo != 1) ||
        ngroups < 1 || !group_col)
        return BSLS_E_ARG;
    Plan p;
    p.rows = rows;
    p.cols = cols;
    p.H = H;
    p.halo = halo;
    p.nrb = (rows + H - 1) / H;
    p.G = ngroups;
    p.nslots = (H + halo + TILE_T - 1) / TILE_T;
    p.indptr = indptr;
    p.indices = indices;
    p.gc = group_col;
    if (p.nslots + 1 > BSLS_TILE_MAXSLOTS) return BSLS_E_ARG;
    if (group_col[0] != 0 || group_col[ngroups] != cols) return BSLS_E_ARG;
    for (int64_t g = 0; g < ngroups; ++g) {
        const int64_t w = group_col[g + 1] - group_col[g];
        if (w < 1 || w > (1 << 24)) return BSLS_E_ARG;   // non-empty, 24-bit offsets
    }
    if (indptr[0] != 0) return BSLS_E_ARG;
    p.gmap.resize(cols);
    for (int64_t g = 0; g < ngroups; ++g)
        for (int64_t j = group_col[g]; j < group_col[g + 1]; ++j) p.gmap[j] = (int32_t)g;
    for (int64_t i = 0; i < rows; ++i)
        if (indptr[i + 1] < indptr[i]) return BSLS_E_ARG;
    for (int64_t k = 0; k < indptr[rows]; ++k)
        if (indices[k] < 0 || indices[k] >= cols) return BSLS_E_ARG;
    // pass 1: quads per wave stream
    const int64_t nwav = p.nrb * ngroups * 16;
    std::vector<int64_t> wq(nwav, 0);
    parallel_blocks(p.nrb, [&](int64_t rb) {
        std::vector<int64_t> cnt;
        count_block(p, rb, cnt);
        for (int64_t g = 0; g < ngroups; ++g)
            for (int w = 0; w < 16; ++w) {
                int64_t mx = 0;
                for (int l = 0; l < 64; ++l) mx = std::max(mx, cnt[(size_t)g * TILE_T + w * 64 + l]);
                wq[(rb * ngroups + g) * 16 + w] = (mx + 3) / 4 * 64;
            }
    });
    int64_t total = 0;
    for (int64_t s = 0; s < nwav; ++s) total += wq[s];
    const int64_t nquads = total;
    if (!wave_off_out) return nquads;
    if (!ent_out || nquads_cap < nquads || (data && !val_out)) return BSLS_E_ARG;
    wave_off_out[0] = 0;
    for (int64_t s = 0; s < nwav; ++s) wave_off_out[s + 1] = wave_off_out[s] + wq[s];
    const uint32_t dummy = (uint32_t)p.nslots << 24;
    // pass 2: bucket, sort by column, scatter into the quads
    parallel_blocks(p.nrb, [&](int64_t rb) {
        std::vector<int64_t> cnt;
        count_block(p, rb, cnt);
        const size_t nb = (size_t)ngroups * TILE_T;
        std::vector<int64_t> off(nb + 1, 0);
        for (size_t k = 0; k < nb; ++k) off[k + 1] = off[k] + cnt[k];
        std::vector<uint64_t> key(off[nb]);
        std::vector<double> val(data ? off[nb] : 0);
        std::vector<int64_t> cur(off.begin(), off.end() - 1);
        const int64_t r0 = rb * p.H;
        for (int64_t i = r0; i < block_end(p, rb); ++i) {
            const int64_t lr = i - r0;
            const int t = (int)(lr % TILE_T);
            const uint64_t slot = (uint64_t)(lr / TILE_T);
            for (int64_t k = p.indptr[i]; k < p.indptr[i + 1]; ++k) {
                const int32_t c = p.indices[k];
                const int64_t g = p.gmap[c];
                const int64_t pos = cur[(size_t)g * TILE_T + t]++;
                key[pos] = ((uint64_t)(c - p.gc[g]) << 8) | slot;   // column, then slot
                if (data) val[pos] = data[k];
            }
        }
        std::vector<int64_t> perm;
        for (int64_t g = 0; g < ngroups; ++g) {
            for (int w = 0; w < 16; ++w) {
                const int64_t s = (rb * ngroups + g) * 16 + w;
                const int64_t base = wave_off_out[s];
                for (int64_t q = base; q < wave_off_out[s + 1]; ++q)
                    for (int j = 0; j < 4; ++j) {
                        ent_out[4 * q + j] = dummy;
                        if (data) val_out[4 * q + j] = 0.0;
                    }
                for (int l = 0; l < 64; ++l) {
                    const size_t bk = (size_t)g * TILE_T + w * 64 + l;
                    const int64_t a = off[bk], e = off[bk + 1];
                    perm.resize(e - a);
                    for (int64_t k = a; k < e; ++k) perm[k - a] = k;
                    std::sort(perm.begin(), perm.end(),
                              [&](int64_t x, int64_t y) { return key[x] < key[y]; });
                    for (int64_t k = 0; k < e - a; ++k) {
                        const int64_t q = base + (k >> 2) * 64 + l;
                        const uint64_t kk = key[perm[k]];
                        ent_out[4 * q + (k & 3)] = (uint32_t)((kk & 0xFF) << 24) | (uint32_t)(kk >> 8);
                        if (data) val_out[4 * q + (k & 3)] = val[perm[k]];
                    }
                }
            }
        }
    });
    return nquads;
}

// ---------------------------------------------------------------------------
// Layout 1 ("dealt", include/bsls_hip.h): per tile (rb, g) the entries sorted
// by (column, local row), packed greedily into 64-lane instructions whose
// columns stay within base + 65535, padded to whole quad-steps (64
// instructions: 4 slots x 16 waves).

namespace {

struct DealtEnt {
    uint64_t key;   // column offset in the group << 16 | local row
    double v;
};

// the tile's sorted entries (values only when data != NULL)
void dealt_collect(const Plan &p, const double *data, int64_t rb, std::vector<std::vector<DealtEnt>> &out) {
    out.assign((size_t)p.G, {});
    const int64_t r0 = rb * p.H;
    for (int64_t i = r0; i < block_end(p, rb); ++i) {
        const uint64_t lr = (uint64_t)(i - r0);
        for (int64_t k = p.indptr[i]; k < p.indptr[i + 1]; ++k) {
            const int32_t c = p.indices[k];
            const int64_t g = p.gmap[c];
            out[(size_t)g].push_back({((uint64_t)(c - p.gc[g]) << 16) | lr, data ? data[k] : 0.0});
        }
    }
    for (auto &v : out)
        std::sort(v.begin(), v.end(),
                  [](const DealtEnt &a, const DealtEnt &b) { return a.key < b.key; });
}

// instruction starts of a sorted tile (greedy: <= 64 entries, column span <= span)
void dealt_insts(const std::vector<DealtEnt> &e, std::vector<int64_t> &st, uint64_t span) {
    st.clear();
    size_t i = 0;
    while (i < e.size()) {
        st.push_back((int64_t)i);
        const uint64_t base = e[i].key >> 16;
        size_t j = i + 1;
        while (j < e.size() && j - i < 64 && (e[j].key >> 16) - base <= span) ++j;
        i = j;
    }
    st.push_back((int64_t)e.size());
}

int bit_width(int64_t v) {
    int b = 0;
    while (v > 0) {
        ++b;
        v >>= 1;
    }
    return b;
}

// layout 1 (packed == false) or 2 (3-byte entries, include/bsls_hip.h)
int64_t build_dealt(int64_t rows, int64_t cols, const int64_t *indptr, const int32_t *indices,
                    const double *data, int64_t H, int64_t halo, int64_t ngroups,
                    const int64_t *group_col, int64_t *wave_off_out, uint32_t *ent_out,
                    int32_t *base_out, double *val_out, int64_t nquads_cap, bool packed);

}  // namespace

extern "C" int64_t bsls_tiles_build_dealt(int64_t rows, int64_t cols, const int64_t *indptr,
                                          const int32_t *indices, const double *data, int64_t H,
                                          int64_t halo, int64_t ngroups, const int64_t *group_col,
                                          int64_t *wave_off_out, uint32_t *ent_out,
                                          int32_t *base_out, double *val_out,
                                          int64_t nquads_cap) {
    return build_dealt(rows, cols, indptr, indices, data, H, halo, ngroups, group_col,
                       wave_off_out, ent_out, base_out, val_out, nquads_cap, false);
}

extern "C" int64_t bsls_tiles_build_dealt3(int64_t rows, int64_t cols, const int64_t *indptr,
                                           const int32_t *indices, const double *data, int64_t H,
                                           int64_t halo, int64_t ngroups, const int64_t *group_col,
                                           int64_t *wave_off_out, uint32_t *ent_out,
                                           int32_t *base_out, double *val_out,
                                           int64_t nquads_cap) {
    return build_dealt(rows, cols, indptr, indices, data, H, halo, ngroups, group_col,
                       wave_off_out, ent_out, base_out, val_out, nquads_cap, true);
}

namespace {

int64_t build_dealt(int64_t rows, int64_t cols, const int64_t *indptr, const int32_t *indices,
                    const double *data, int64_t H, int64_t halo, int64_t ngroups,
                    const int64_t *group_col, int64_t *wave_off_out, uint32_t *ent_out,
                    int32_t *base_out, double *val_out, int64_t nquads_cap, bool packed) {
    if (rows < 1 || cols < 1 || !indptr || !indices || H < 64 || (halo != 0 && halo != 1) ||
        ngroups < 1 || !group_col || H + halo + 1 > 65536)
        return BSLS_E_ARG;
    // packed: 24-bit entries, local row (rbits, the dummy row H + halo
    // included) above the column offset (cbits = 24 - rbits)
    const int rbits = bit_width(H + halo), cbits = 24 - rbits;
    if (packed && cbits < 6) return BSLS_E_ARG;
    const uint64_t span = packed ? ((1ull << cbits) - 1) : 65535ull;
    Plan p;
    p.rows = rows;
    p.cols = cols;
    p.H = H;
    p.halo = halo;
    p.nrb = (rows + H - 1) / H;
    p.G = ngroups;
    p.nslots = 0;
    p.indptr = indptr;
    p.indices = indices;
    p.gc = group_col;
    if (group_col[0] != 0 || group_col[ngroups] != cols) return BSLS_E_ARG;
    for (int64_t g = 0; g < ngroups; ++g) {
        const int64_t w = group_col[g + 1] - group_col[g];
        if (w < 1 || w > INT32_MAX) return BSLS_E_ARG;   // int32 bases
    }
    if (indptr[0] != 0) return BSLS_E_ARG;
    p.gmap.resize(cols);
    for (int64_t g = 0; g < ngroups; ++g)
        for (int64_t j = group_col[g]; j < group_col[g + 1]; ++j) p.gmap[j] = (int32_t)g;
    for (int64_t i = 0; i < rows; ++i)
        if (indptr[i + 1] < indptr[i]) return BSLS_E_ARG;
    for (int64_t k = 0; k < indptr[rows]; ++k)
        if (indices[k] < 0 || indices[k] >= cols) return BSLS_E_ARG;
    // pass 1: quad-steps per tile
    const int64_t ntiles = p.nrb * ngroups;
    std::vector<int64_t> qs(ntiles, 0);
    parallel_blocks(p.nrb, [&](int64_t rb) {
        std::vector<std::vector<DealtEnt>> e;
        std::vector<int64_t> st;
        dealt_collect(p, nullptr, rb, e);
        for (int64_t g = 0; g < ngroups; ++g) {
            dealt_insts(e[(size_t)g], st, span);
            const int64_t ni = (int64_t)st.size() - 1;
            qs[rb * ngroups + g] = (ni + 63) / 64;
        }
    });
    int64_t total = 0;
    for (int64_t t = 0; t < ntiles; ++t) total += qs[t];
    const int64_t nquads = total * 1024;
    if (!wave_off_out) return nquads;
    if (!ent_out || !base_out || nquads_cap < nquads || (data && !val_out)) return BSLS_E_ARG;
    wave_off_out[0] = 0;
    for (int64_t t = 0; t < ntiles; ++t) wave_off_out[t + 1] = wave_off_out[t] + qs[t];
    const int rshift = packed ? cbits : 16;
    const uint32_t dummy = (uint32_t)(H + halo) << rshift;
    // pass 2: fill (packed: each tile in the 4-per-lane form first, then 3
    // uint32 per lane: e0 | e1 << 24, e1 >> 8 | e2 << 16, e2 >> 16 | e3 << 8)
    parallel_blocks(p.nrb, [&](int64_t rb) {
        std::vector<std::vector<DealtEnt>> e;
        std::vector<int64_t> st;
        std::vector<uint32_t> tmp;
        dealt_collect(p, data, rb, e);
        for (int64_t g = 0; g < ngroups; ++g) {
            const auto &E = e[(size_t)g];
            dealt_insts(E, st, span);
            const int64_t t = rb * ngroups + g, q0 = wave_off_out[t];
            const int64_t nslot = (wave_off_out[t + 1] - q0) * 64;   // instructions incl. padding
            const int64_t ni = (int64_t)st.size() - 1;
            uint32_t *eo = ent_out + 4 * q0 * 1024;
            if (packed) {
                tmp.assign((size_t)(4 * (wave_off_out[t + 1] - q0) * 1024), 0u);
                eo = tmp.data();
            }
            for (int64_t k = 0; k < nslot; ++k) {
                const int64_t w = k % 16, j = (k / 16) % 4, q = q0 + k / 64;
                const int64_t qi = (q * 16 + w) * 64;           // uint4 index of lane 0
                uint32_t base = 0;
                int64_t a = 0, b = 0;
                if (k < ni) {
                    a = st[(size_t)k];
                    b = st[(size_t)k + 1];
                    base = (uint32_t)(E[(size_t)a].key >> 16);
                }
                base_out[(q * 16 + w) * 4 + j] = (int32_t)base;
                for (int64_t l = 0; l < 64; ++l) {
                    const int64_t u = 4 * (qi + l) + j;
                    const int64_t ul = u - 4 * q0 * 1024;       // within the tile
                    if (a + l < b) {
                        const DealtEnt &d = E[(size_t)(a + l)];
                        eo[ul] = (uint32_t)(d.key & 0xFFFF) << rshift |
                                 (uint32_t)((d.key >> 16) - base);
                        if (data) val_out[u] = d.v;
                    } else {
                        eo[ul] = dummy;
                        if (data) val_out[u] = 0.0;
                    }
                }
            }
            if (packed) {
                const int64_t nl = (wave_off_out[t + 1] - q0) * 1024;   // lanes of the tile
                uint32_t *po = ent_out + 3 * q0 * 1024;
                for (int64_t i = 0; i < nl; ++i) {
                    const uint32_t e0 = tmp[4 * i], e1 = tmp[4 * i + 1], e2 = tmp[4 * i + 2],
                                   e3 = tmp[4 * i + 3];
                    po[3 * i] = e0 | (e1 << 24);
                    po[3 * i + 1] = (e1 >> 8) | (e2 << 16);
                    po[3 * i + 2] = (e2 >> 16) | (e3 << 8);
                }
            }
        }
    });
    return nquads;
}

}  // namespace
