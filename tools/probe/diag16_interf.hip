// Does work on the OTHER SIMDs of a CU slow the BCR pivot wave?  Wave 0 of a
// 512-thread workgroup (8 waves, two per SIMD: waves w and w + 4 share one)
// times R repetitions of the in-register 16x16 factor + inverse (diag16's
// arithmetic), while waves 1-3 and 5-7 (SIMDs 1-3) run a helper loop until
// wave 0 is done; wave 4 (wave 0's SIMD mate) stays idle, as in
// bcr_level_kernel's factor windows.  Helper modes: 0 idle, 1 fp64 MFMA
// chains on registers, 2 LDS reads / writes, 3 fp64 MFMA tile products fed
// from LDS (the level kernel's helper work), 4 fp64 VALU FMAs.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/diag16_interf.hip -o tools/probe/diag16_interf
#include <hip/hip_runtime.h>
#include <cstdio>
#include <utility>
#include <vector>

__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ double rsqrt_n(double d) {
    double y = __builtin_amdgcn_rsq(d);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const double hy = 0.5 * d * y;
        y = fma(y, fma(-hy, y, 0.5), y);
    }
    return y;
}
__device__ __forceinline__ double row_bcast(double v, int l) {
#define P_BC(n) case n: return __builtin_amdgcn_mov_dpp(v, 0x150 + n, 0xf, 0xf, true);
    switch (l) {
        P_BC(0) P_BC(1) P_BC(2) P_BC(3) P_BC(4) P_BC(5) P_BC(6) P_BC(7)
        P_BC(8) P_BC(9) P_BC(10) P_BC(11) P_BC(12) P_BC(13) P_BC(14)
        default: return __builtin_amdgcn_mov_dpp(v, 0x15f, 0xf, 0xf, true);
    }
#undef P_BC
}
#define P_FMAC(n)                                                                                      \
    case n:                                                                                            \
        if (NOP)                                                                                       \
            asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:" #n " row_mask:0xf bank_mask:0xf" \
                         : "+v"(acc) : "v"(src), "v"(mul));                                            \
        else                                                                                           \
            asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #n " row_mask:0xf bank_mask:0xf"   \
                         : "+v"(acc) : "v"(src), "v"(mul));                                            \
        break;
template <bool NOP>
__device__ __forceinline__ void fmac_bc(double& acc, double src, double mul, int l) {
    switch (l) {
        P_FMAC(0) P_FMAC(1) P_FMAC(2) P_FMAC(3) P_FMAC(4) P_FMAC(5) P_FMAC(6) P_FMAC(7)
        P_FMAC(8) P_FMAC(9) P_FMAC(10) P_FMAC(11) P_FMAC(12) P_FMAC(13) P_FMAC(14) P_FMAC(15)
        default: break;
    }
}
template <int K, int... J>
__device__ __forceinline__ void upd(double (&a)[16], double nt, std::integer_sequence<int, J...>) {
    (fmac_bc<J == 0>(a[K + 1 + J], a[K], nt, K + 1 + J), ...);
}
template <int K, int... P>
__device__ __forceinline__ void xrow(const double (&a)[16], const double (&x)[16], double& u0, double& u1,
                                     std::integer_sequence<int, P...>) {
    ((P & 1 ? fmac_bc<false>(u1, a[P], x[P], K) : fmac_bc<P == 0>(u0, a[P], x[P], K)), ...);
}
template <int K>
__device__ __forceinline__ void step(double (&a)[16], double (&x)[16], int i) {
    const double d = row_bcast(a[K], K);
    const double rinv = rsqrt_n(d);
    const double lk = a[K] * rinv;
    const double nt = -(lk * rinv);
    upd<K>(a, nt, std::make_integer_sequence<int, 15 - K>{});
    a[K] = lk;
    double u0 = 0.0, u1 = 0.0;
    xrow<K>(a, x, u0, u1, std::make_integer_sequence<int, K>{});
    x[K] = ((K == i ? 1.0 : 0.0) - (u0 + u1)) * rinv;
    if constexpr (K < 15) step<K + 1>(a, x, i);
}

typedef double v4d __attribute__((ext_vector_type(4)));
template <int H>
__global__ __launch_bounds__(512) void interf(const double* A, double* out, unsigned long long* cyc, int reps) {
    __shared__ double lds[64 * 65 * 2];
    __shared__ int done;
    const int wave = threadIdx.x >> 6, i = threadIdx.x & 63;
    if (threadIdx.x == 0) done = 0;
    for (int e = threadIdx.x; e < 64 * 65 * 2; e += 512) lds[e] = 1e-3 * (e % 977);
    __syncthreads();
    if (wave == 0) {
        double a0[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) a0[j] = (i < 16 && j <= i) ? A[i * 16 + j] : (i == j ? 1.0 : 0.0);
        double sink = 0.0;
        __builtin_amdgcn_s_setprio(2);
        const unsigned long long t0 = stamp();
        for (int r = 0; r < reps; ++r) {
            double a[16], x[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) { a[j] = a0[j] + sink * 1e-300; x[j] = 0.0; }
            step<0>(a, x, i);
            sink += a[15] + x[15];
        }
        const unsigned long long t1 = stamp();
        __builtin_amdgcn_s_setprio(0);
        out[i] = sink;
        if (i == 0) cyc[H] = t1 - t0;
        __hip_atomic_store(&done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return;
    }
    if (H == 0 || wave == 4) return;
    v4d acc = {0, 0, 0, 0};
    double v = lds[i], w = 0.0;
    const int ii = i & 15, kk = i >> 4;
    // bounded: a lost 'done' store cannot hang the box
    for (int rounds = 0; rounds < (1 << 20); ++rounds) {
        if (__hip_atomic_load(&done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0) break;
        for (int it = 0; it < 16; ++it) {
            if constexpr (H == 1) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, acc, 0, 0, 0);
            if constexpr (H == 2) {
                lds[(wave * 64 + i + it * 7) % (64 * 65)] = v;
                v = lds[(i * 65 + it) % (64 * 65)];
            }
            if constexpr (H == 3) {   // one 16x16 tile, one 16-deep k chunk, operands from LDS
                const int k0 = 16 * (it & 3);
                double av[4], bv[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    av[j] = lds[(16 * (wave & 3) + ii) * 65 + k0 + 4 * j + kk];
                    bv[j] = lds[64 * 65 + (k0 + 4 * j + kk) * 65 + ii];
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[j], bv[j], acc, 0, 0, 0);
            }
            if constexpr (H == 4) {
                w = fma(v, w, 1.0);
                v = fma(w, v, 0.5);
            }
        }
    }
    out[64 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3] + v + w;
}

int main() {
    std::vector<double> A(256);
    for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) A[r * 16 + c] = (r == c ? 20.0 : 0.0) + 1.0 / (1 + r + c);
    double *dA, *dout;
    unsigned long long* dc;
    hipMalloc(&dA, 256 * 8);
    hipMalloc(&dout, 1024 * 8);
    hipMalloc(&dc, 16 * 8);
    hipMemcpy(dA, A.data(), 256 * 8, hipMemcpyHostToDevice);
    hipMemset(dc, 0, 16 * 8);
    const int reps = 500;
    const char* hn[] = {"idle", "fp64 MFMA (registers)", "LDS reads/writes", "fp64 MFMA tiles from LDS",
                        "fp64 VALU FMAs"};
    for (int pass = 0; pass < 2; ++pass) {
        interf<0><<<1, 512>>>(dA, dout, dc, reps);
        interf<1><<<1, 512>>>(dA, dout, dc, reps);
        interf<2><<<1, 512>>>(dA, dout, dc, reps);
        interf<3><<<1, 512>>>(dA, dout, dc, reps);
        interf<4><<<1, 512>>>(dA, dout, dc, reps);
        if (hipDeviceSynchronize() != hipSuccess) return 1;
    }
    unsigned long long c[16];
    hipMemcpy(c, dc, 16 * 8, hipMemcpyDeviceToHost);
    for (int h = 0; h < 5; ++h)
        printf("wave 0's factor, waves 1-3 + 5-7 running %-26s %8.0f cycles/factor\n", hn[h], (double)c[h] / reps);
    return 0;
}
