// Which SIMD does each wave of a 512-thread workgroup run on (gfx950 HW_ID:
// WAVE_ID [3:0], SIMD_ID [5:4], CU_ID [11:8])?  Prints the map of a few
// workgroups.  hipcc --offload-arch=gfx950 -O2 simd_probe.hip -o simd_probe
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(512) void probe(int* out) {
    const unsigned id = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_ID, 32 bits
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = (int)id;
}
int main() {
    const int nb = 16;
    int* d; hipMalloc(&d, nb * 8 * sizeof(int));
    hipLaunchKernelGGL(probe, dim3(nb), dim3(512), 0, 0, d);
    int h[nb * 8];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int b = 0; b < nb; ++b) {
        printf("wg %2d:", b);
        for (int w = 0; w < 8; ++w) printf("  w%d simd %d cu %2d wid %d", w, (h[b * 8 + w] >> 4) & 3, (h[b * 8 + w] >> 8) & 15, h[b * 8 + w] & 15);
        printf("\n");
    }
    return 0;
}
