// PMC calibration (MI355X_MICROARCH.md "HBM": FETCH_SIZE reads half the bytes
// of 16-B-per-lane streaming reads; other widths uncalibrated): kernels that
// move a known byte count in the access widths the BB kernels use, one launch
// each, named by width, so `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
// rows can be divided by the known bytes.  Buffer 256 MiB per launch, each
// launch on a buffer the previous ones did not touch (L2-cold; MALL-cold for
// the first pass over it).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("hip %d line %d\n", e_, __LINE__); return 1; } } while (0)

__global__ void rd16(const double2 *__restrict__ a, size_t n, double *out) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[i].x + a[i].y;
    if (s == 12345.678) out[0] = s;
}
__global__ void rd8(const double *__restrict__ a, size_t n, double *out) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[i];
    if (s == 12345.678) out[0] = s;
}
__global__ void wr8(double *__restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = (double)i;
}
__global__ void wr16(double2 *__restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_double2((double)i, 1.0);
}

int main() {
    const size_t bytes = (size_t)256 << 20;
    double *buf[6], *out;
    for (int k = 0; k < 6; ++k) {
        CK(hipMalloc(&buf[k], bytes));
        CK(hipMemset(buf[k], 0, bytes));
    }
    CK(hipMalloc(&out, 64));
    // evict: touch a 1 GiB scratch between the fills and the timed reads
    double *scr;
    CK(hipMalloc(&scr, (size_t)1 << 30));
    CK(hipMemset(scr, 1, (size_t)1 << 30));
    CK(hipDeviceSynchronize());
    const int grid = 4096, blk = 256;
    rd16<<<grid, blk>>>((const double2 *)buf[0], bytes / 16, out);   // 256 MiB read, 16 B/lane
    CK(hipMemset(scr, 2, (size_t)1 << 30));
    rd8<<<grid, blk>>>(buf[1], bytes / 8, out);                       // 256 MiB read, 8 B/lane
    CK(hipMemset(scr, 3, (size_t)1 << 30));
    wr8<<<grid, blk>>>(buf[2], bytes / 8);                            // 256 MiB written, 8 B/lane
    CK(hipMemset(scr, 4, (size_t)1 << 30));
    wr16<<<grid, blk>>>((double2 *)buf[3], bytes / 16);               // 256 MiB written, 16 B/lane
    CK(hipDeviceSynchronize());
    printf("fetch_calib: 4 launches of 262144 KiB each (rd16 rd8 wr8 wr16)\n");
    return 0;
}
