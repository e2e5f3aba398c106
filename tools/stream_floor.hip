// stream_floor.hip -- what an in-place pass over C2's 3.2M doubles (25.6 MB
// read + 25.6 MB written) costs per HBM-fed launch on this chip, for the
// projection's roofline discussion: 16 distinct buffers (410
// MB, beyond the Infinity Cache) scaled back to back between two events, as
// bench.py's proj leg times the projection.  Forms: one double per thread;
// 16 B per thread; 16 B with write-through (sc1) stores; U x 16 B per
// thread, every load issued before the first store.
//   hipcc --offload-arch=gfx950 -O3 -o tools/stream_floor tools/stream_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__global__ void scale1(double *y, long n, double a) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] *= a;
}

typedef double d2 __attribute__((ext_vector_type(2)));

template <int U, int AUX>
__global__ __launch_bounds__(256) void scaleU(double *y, long n, double a) {
    const long q0 = ((long)blockIdx.x * blockDim.x * U + threadIdx.x);
    d2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long q = q0 + (long)u * blockDim.x;
        v[u] = (2 * q + 1 < n) ? reinterpret_cast<const d2 *>(y)[q] : d2{0.0, 0.0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long q = q0 + (long)u * blockDim.x;
        if (2 * q + 1 < n) {
            const d2 r = v[u] * a;
            if (AUX)
                __builtin_nontemporal_store(r, reinterpret_cast<d2 *>(y) + q);
            else
                reinterpret_cast<d2 *>(y)[q] = r;
        }
    }
}

// the window structure a segmented projection would have: each wave a fixed
// 512-entry window (+64 overhang read, not written), loaded coalesced, turned
// into 8 consecutive entries per lane through LDS and back, one segmented
// scan step per lane's run (a stand-in for one pass), stored coalesced
__global__ __launch_bounds__(256) void window_skel(double *y, long n, double a) {
    __shared__ double buf[4][576 + 8];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long w = (long)blockIdx.x * 4 + wv;
    const long b0 = w * 512;
    if (b0 >= n) return;
    double t[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) {
        const long i = b0 + 64 * e + lane;
        t[e] = i < n ? y[i] : 0.0;
    }
    double *B = buf[wv];
#pragma unroll
    for (int e = 0; e < 9; ++e) B[64 * e + lane] = t[e];
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = B[8 * lane + k];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
    // one wave-wide inclusive scan of the lane sums (6 steps), as a pass costs
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double u = __shfl_up(s, o, 64);
        if (lane >= o) s += u;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) B[8 * lane + k] = v[k] * a + s * 1e-300;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const long i = b0 + 64 * e + lane;
        if (i < n) __builtin_nontemporal_store(B[64 * e + lane], y + i);
    }
}

int main() {
    const long n = 3200000;
    const int B = 16;
    std::vector<double *> ys(B);
    for (auto &p : ys) {
        CK(hipMalloc(&p, n * 8));
        CK(hipMemset(p, 0, n * 8));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) -> int {
        std::vector<float> t;
        for (int rep = 0; rep < 7; ++rep) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            for (int b = 0; b < B; ++b) launch(ys[b]);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms * 1000.f / B);
        }
        std::sort(t.begin(), t.end());
        printf("%-28s %7.2f us/launch (min %.2f)  %.2f TB/s\n", name, t[3], t[0],
               16.0 * n / (t[3] * 1e-6) / 1e12);
        return 0;
    };
    run("1 double / thread", [&](double *y) { scale1<<<(n + 255) / 256, 256>>>(y, n, 1.0000001); });
    run("16 B / thread", [&](double *y) {
        scaleU<1, 0><<<(n / 2 + 255) / 256, 256>>>(y, n, 1.0000001);
    });
    run("16 B / thread, nt stores", [&](double *y) {
        scaleU<1, 1><<<(n / 2 + 255) / 256, 256>>>(y, n, 1.0000001);
    });
    run("4 x 16 B / thread", [&](double *y) {
        scaleU<4, 0><<<(n / 2 + 1023) / 1024, 256>>>(y, n, 1.0000001);
    });
    run("4 x 16 B / thread, nt", [&](double *y) {
        scaleU<4, 1><<<(n / 2 + 1023) / 1024, 256>>>(y, n, 1.0000001);
    });
    run("8 x 16 B / thread", [&](double *y) {
        scaleU<8, 0><<<(n / 2 + 2047) / 2048, 256>>>(y, n, 1.0000001);
    });
    run("window 512 + LDS both ways", [&](double *y) {
        window_skel<<<(n / 512 + 4) / 4, 256>>>(y, n, 1.0000001);
    });
    return 0;
}
