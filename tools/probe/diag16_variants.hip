// Cycle costs of the BCR pivot wave's building blocks on one wave (gfx950),
// and of variants of diag16's per-pivot instruction stream:
//   micro: independent / dependent v_fma_f64, v_fmac_f64_dpp row_newbcast,
//          v_rsq_f64
//   diag16: V0 as shipped (two Newton steps, x_K = (delta - u0 - u1) rinv);
//           V1 one Newton step; V2 the identity column carried in x (x_K =
//           (x_K - u0 - u1) rinv, the chain subtracting with a negated DPP
//           source); V3 both.
// Every variant's L and X are compared with V0's (max abs difference).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/diag16_variants.hip -o tools/probe/diag16_variants
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <utility>
#include <vector>

__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
template <int NEWTON>
__device__ __forceinline__ double rsqrt_n(double d) {
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
#pragma unroll
    for (int it = 0; it < NEWTON; ++it) y = fma(y, fma(-(h * y), y, 0.5), y);
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
// acc += src[lane n] * mul (NEG: acc -= ...)
#define P_FMAC(n)                                                                                          \
    case n:                                                                                                \
        if (NOP && NEG)                                                                                    \
            asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:" #n " row_mask:0xf bank_mask:0xf" \
                         : "+v"(acc) : "v"(src), "v"(mul));                                                \
        else if (NOP)                                                                                      \
            asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:" #n " row_mask:0xf bank_mask:0xf" \
                         : "+v"(acc) : "v"(src), "v"(mul));                                                \
        else if (NEG)                                                                                      \
            asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:" #n " row_mask:0xf bank_mask:0xf"      \
                         : "+v"(acc) : "v"(src), "v"(mul));                                                \
        else                                                                                               \
            asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #n " row_mask:0xf bank_mask:0xf"       \
                         : "+v"(acc) : "v"(src), "v"(mul));                                                \
        break;
template <bool NOP, bool NEG = false>
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
template <int K, bool NEG, int... P>
__device__ __forceinline__ void xrow(const double (&a)[16], const double (&x)[16], double& u0, double& u1,
                                     std::integer_sequence<int, P...>) {
    ((P & 1 ? fmac_bc<false, NEG>(u1, a[P], x[P], K) : fmac_bc<P == 0, NEG>(u0, a[P], x[P], K)), ...);
}
// V: bit 0 one Newton step, bit 1 identity column carried in x
template <int V, int K>
__device__ __forceinline__ void step(double (&a)[16], double (&x)[16], int i) {
    constexpr bool kId = V & 2;
    const double d = row_bcast(a[K], K);
    const double rinv = rsqrt_n<(V & 1) ? 1 : 2>(d);
    const double lk = a[K] * rinv;
    const double nt = -(lk * rinv);
    upd<K>(a, nt, std::make_integer_sequence<int, 15 - K>{});
    a[K] = lk;
    if constexpr (kId) {
        double u0 = x[K], u1 = 0.0;   // delta_Ki - sum_p L_Kp x_p
        xrow<K, true>(a, x, u0, u1, std::make_integer_sequence<int, K>{});
        x[K] = (u0 + u1) * rinv;
    } else {
        double u0 = 0.0, u1 = 0.0;
        xrow<K, false>(a, x, u0, u1, std::make_integer_sequence<int, K>{});
        x[K] = ((K == i ? 1.0 : 0.0) - (u0 + u1)) * rinv;
    }
    if constexpr (K < 15) step<V, K + 1>(a, x, i);
}

template <int V>
__global__ __launch_bounds__(64) void fac(const double* A, double* out, unsigned long long* cyc, int reps) {
    const int i = threadIdx.x;
    double a0[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) a0[j] = (i < 16 && j <= i) ? A[i * 16 + j] : (i == j ? 1.0 : 0.0);
    double sink = 0.0, a[16], x[16];
    const unsigned long long t0 = stamp();
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            a[j] = a0[j] + sink * 1e-300;
            x[j] = (V & 2) ? (j == i ? 1.0 : 0.0) : 0.0;
        }
        step<V, 0>(a, x, i);
        sink += a[15] + x[15];
    }
    const unsigned long long t1 = stamp();
    if (i < 16) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            out[V * 512 + i * 16 + j] = a[j];
            out[V * 512 + 256 + j * 16 + i] = x[j];
        }
    }
    if (i == 0) cyc[V] = t1 - t0;
    if (sink == 12345.0) out[4096] = sink;
}

// micro: M 0 independent fma (8 chains), 1 dependent fma chain, 2 independent fmac_dpp (8 chains),
// 3 dependent fmac_dpp chain, 4 rsq chain
template <int M>
__global__ __launch_bounds__(64) void micro(double* out, unsigned long long* cyc, int reps) {
    double c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = 1e-3 * (threadIdx.x + j);
    const double m = 0.999999, s = 1e-9;
    const unsigned long long t0 = stamp();
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if constexpr (M == 0) {
#pragma unroll
                for (int j = 0; j < 8; ++j) c[j] = fma(c[j], m, s);
            } else if constexpr (M == 1) {
#pragma unroll
                for (int j = 0; j < 8; ++j) c[0] = fma(c[0], m, s);
            } else if constexpr (M == 2) {
#pragma unroll
                for (int j = 0; j < 8; ++j) fmac_bc<false>(c[j], c[(j + 1) & 7], s, 3);
            } else if constexpr (M == 3) {
#pragma unroll
                for (int j = 0; j < 8; ++j) fmac_bc<true>(c[0], c[1], s, 3);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) c[0] = __builtin_amdgcn_rsq(c[0] + 1.0);
            }
        }
    }
    const unsigned long long t1 = stamp();
    double t = 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) t += c[j];
    out[threadIdx.x] = t;
    if (threadIdx.x == 0) cyc[8 + M] = t1 - t0;
}

int main() {
    std::vector<double> A(256);
    for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) A[r * 16 + c] = (r == c ? 20.0 : 0.0) + 1.0 / (1 + r + c);
    double *dA, *dout;
    unsigned long long* dc;
    hipMalloc(&dA, 256 * 8);
    hipMalloc(&dout, 4100 * 8);
    hipMalloc(&dc, 16 * 8);
    hipMemcpy(dA, A.data(), 256 * 8, hipMemcpyHostToDevice);
    const int reps = 500, mreps = 200;
    for (int pass = 0; pass < 2; ++pass) {
        fac<0><<<1, 64>>>(dA, dout, dc, reps);
        fac<1><<<1, 64>>>(dA, dout, dc, reps);
        fac<2><<<1, 64>>>(dA, dout, dc, reps);
        fac<3><<<1, 64>>>(dA, dout, dc, reps);
        micro<0><<<1, 64>>>(dout, dc, mreps);
        micro<1><<<1, 64>>>(dout, dc, mreps);
        micro<2><<<1, 64>>>(dout, dc, mreps);
        micro<3><<<1, 64>>>(dout, dc, mreps);
        micro<4><<<1, 64>>>(dout, dc, mreps);
        if (hipDeviceSynchronize() != hipSuccess) return 1;
    }
    unsigned long long c[16];
    std::vector<double> o(4100);
    hipMemcpy(c, dc, 16 * 8, hipMemcpyDeviceToHost);
    hipMemcpy(o.data(), dout, 4100 * 8, hipMemcpyDeviceToHost);
    const char* vn[] = {"shipped (2 Newton, delta select)", "1 Newton", "identity column in x", "1 Newton + identity column"};
    for (int v = 0; v < 4; ++v) {
        double dl = 0.0, dx = 0.0;
        for (int e = 0; e < 256; ++e) {
            dl = std::fmax(dl, std::fabs(o[v * 512 + e] - o[e]));
            dx = std::fmax(dx, std::fabs(o[v * 512 + 256 + e] - o[256 + e]));
        }
        printf("diag16 %-34s %7.0f cycles/factor  max|dL| %.2e  max|dX| %.2e\n", vn[v], (double)c[v] / reps, dl, dx);
    }
    const char* mn[] = {"v_fma_f64 independent", "v_fma_f64 dependent", "v_fmac_f64_dpp independent",
                        "v_fmac_f64_dpp dependent (+s_nop 1)", "v_rsq_f64 + v_add dependent"};
    for (int m = 0; m < 5; ++m) printf("%-40s %6.2f cycles/instruction\n", mn[m], (double)c[8 + m] / (mreps * 64.0));
    return 0;
}
