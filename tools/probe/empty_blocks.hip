// Probe: the cost of dispatching workgroups that find the device-side queue count past their range and
// exit at once (the capacity-sized grids of the shading / traversal launches), against a real grid.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(64) void k_exit(const int* __restrict__ count, float* out) {
    const int n = *count;
    if ((int)blockIdx.x * 64 >= n) return;
    out[blockIdx.x * 64 + threadIdx.x] = 1.0f;
}
int main() {
    int* cnt;
    float* out;
    hipMalloc(&cnt, 4);
    hipMalloc(&out, 4ull << 26);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grids[] = {1 << 14, 1 << 17, 1 << 19, 1 << 20};
    for (int g : grids) {
        for (int live : {0, 1}) {
            const int n = live ? g * 64 : 0;
            hipMemcpy(cnt, &n, 4, hipMemcpyHostToDevice);
            hipLaunchKernelGGL(k_exit, dim3(g), dim3(64), 0, 0, cnt, out);
            hipDeviceSynchronize();
            float best = 1e9f;
            for (int r = 0; r < 5; ++r) {
                hipEventRecord(a);
                hipLaunchKernelGGL(k_exit, dim3(g), dim3(64), 0, 0, cnt, out);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                best = ms < best ? ms : best;
            }
            printf("blocks %8d  %s  %.4f ms  (%.2f ns per block)\n", g, live ? "writing" : "empty  ", best, best * 1e6 / g);
        }
    }
    return 0;
}
