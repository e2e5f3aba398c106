// Fixed cost of a launch shaped like the tile kernels (tools/launch_ubench.hip):
// back-to-back launches of a kernel that only clears its LDS and stores one
// double per thread, for several (workgroups x threads, LDS) shapes.
//   hipcc --offload-arch=gfx950 -O3 -o launch_ubench tools/launch_ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void touch(double *out, int lds_doubles) {
    extern __shared__ double lds[];
    for (int i = threadIdx.x; i < lds_doubles; i += blockDim.x) lds[i] = 0.0;
    __syncthreads();
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = lds[threadIdx.x % (lds_doubles > 0 ? lds_doubles : 1)];
}

int main() {
    double *out;
    hipMalloc(&out, (size_t)4096 * 1024 * 8);
    hipFuncSetAttribute((const void *)touch, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    struct Shape { int wg, thr, lds; } shapes[] = {
        {256, 1024, 3126}, {256, 1024, 15626}, {256, 1024, 0}, {512, 1024, 3126},
        {1024, 256, 3126}, {256, 256, 3126}, {256, 64, 0}, {4096, 64, 0}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (auto s : shapes) {
        for (int w = 0; w < 20; ++w) touch<<<s.wg, s.thr, s.lds * 8>>>(out, s.lds);
        hipDeviceSynchronize();
        const int reps = 200;
        hipEventRecord(a);
        for (int r = 0; r < reps; ++r) touch<<<s.wg, s.thr, s.lds * 8>>>(out, s.lds);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("wg %5d x %4d threads, LDS %6d B: %.2f us per launch\n", s.wg, s.thr, s.lds * 8,
               ms * 1e3 / reps);
    }
    return 0;
}
