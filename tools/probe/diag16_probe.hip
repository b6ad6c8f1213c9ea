// Cycle cost of the BCR / dense diagonal 16x16 factor (diag16 in ba_bcr.hip)
// in isolation, one wave: variants without the inverse rows, with one Newton
// step, and two independent factors interleaved (latency vs issue bound).
// s_memtime around R repetitions; prints cycles per factor and per pivot.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <utility>
#include <vector>

__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
template <int NW>
__device__ __forceinline__ double rsqrt_n(double d) {
    double y = __builtin_amdgcn_rsq(d);
#pragma unroll
    for (int it = 0; it < NW; ++it) {
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
// plain-C form of the same update (compiler-visible: it may schedule freely)
template <int K, int... J>
__device__ __forceinline__ void upd_asm(double (&a)[16], double nt, std::integer_sequence<int, J...>) {
    (fmac_bc<J == 0>(a[K + 1 + J], a[K], nt, K + 1 + J), ...);
}
template <int K, int... J>
__device__ __forceinline__ void upd_c(double (&a)[16], double nt, std::integer_sequence<int, J...>) {
    ((a[K + 1 + J] = fma(row_bcast(a[K], K + 1 + J), nt, a[K + 1 + J])), ...);
}
template <int K, int... P>
__device__ __forceinline__ void xrow(const double (&a)[16], const double (&x)[16], double& u0, double& u1,
                                     std::integer_sequence<int, P...>) {
    ((P & 1 ? fmac_bc<false>(u1, a[P], x[P], K) : fmac_bc<P == 0>(u0, a[P], x[P], K)), ...);
}
template <int K, bool XR, int NW, bool CU>
__device__ __forceinline__ void step(double (&a)[16], double (&x)[16], int i) {
    const double d = row_bcast(a[K], K);
    const double rinv = rsqrt_n<NW>(d);
    const double lk = a[K] * rinv;
    const double nt = -(lk * rinv);
    if constexpr (CU) upd_c<K>(a, nt, std::make_integer_sequence<int, 15 - K>{});
    else upd_asm<K>(a, nt, std::make_integer_sequence<int, 15 - K>{});
    a[K] = lk;
    if constexpr (XR) {
        double u0 = 0.0, u1 = 0.0;
        xrow<K>(a, x, u0, u1, std::make_integer_sequence<int, K>{});
        x[K] = ((K == i ? 1.0 : 0.0) - (u0 + u1)) * rinv;
    }
    if constexpr (K < 15) step<K + 1, XR, NW, CU>(a, x, i);
}
// fraction-free (Bareiss) chain: a_ij <- (d_K a_ij - a_iK a_jK) / d_{K-1}, as
// a_ij <- fma(d_K r, a_ij, -(a_jK (a_iK r))) with r = 1 / d_{K-1} one step old
template <int K, int... J>
__device__ __forceinline__ void bar_upd(double (&a)[16], double dr, double s, std::integer_sequence<int, J...>) {
    ((a[K + 1 + J] *= dr), ...);
    (fmac_bc<J == 0>(a[K + 1 + J], a[K], -s, K + 1 + J), ...);
}
template <int K>
__device__ __forceinline__ void bstep(double (&a)[16], double (&piv)[16], double r) {
    const double d = row_bcast(a[K], K);
    piv[K] = d;
    const double s = a[K] * r, dr = d * r;
    if constexpr (K < 15) {
        bar_upd<K>(a, dr, s, std::make_integer_sequence<int, 15 - K>{});
        bstep<K + 1>(a, piv, __builtin_amdgcn_rcp(d));   // (Newton steps off the chain in a real version)
    }
}
// Halley (third-order) rsq refinement: one step, 5 dependent ops
__device__ __forceinline__ double rsqrt_h(double d) {
    const double y = __builtin_amdgcn_rsq(d);
    const double e = fma(-d * y, y, 1.0);
    const double p = fma(0.375, e, 0.5);
    return fma(y, e * p, y);
}
template <int K>
__device__ __forceinline__ void hstep(double (&a)[16], double (&x)[16], int i) {
    const double d = row_bcast(a[K], K);
    const double rinv = rsqrt_h(d);
    const double lk = a[K] * rinv;
    const double nt = -(lk * rinv);
    upd_asm<K>(a, nt, std::make_integer_sequence<int, 15 - K>{});
    a[K] = lk;
    double u0 = 0.0, u1 = 0.0;
    xrow<K>(a, x, u0, u1, std::make_integer_sequence<int, K>{});
    x[K] = ((K == i ? 1.0 : 0.0) - (u0 + u1)) * rinv;
    if constexpr (K < 15) hstep<K + 1>(a, x, i);
}
// two independent factors, steps interleaved
template <int K, int NW>
__device__ __forceinline__ void step2(double (&a)[16], double (&b)[16]) {
    const double da = row_bcast(a[K], K), db = row_bcast(b[K], K);
    const double ra = rsqrt_n<NW>(da), rb = rsqrt_n<NW>(db);
    const double la = a[K] * ra, lb = b[K] * rb;
    const double na = -(la * ra), nb = -(lb * rb);
    upd_asm<K>(a, na, std::make_integer_sequence<int, 15 - K>{});
    upd_asm<K>(b, nb, std::make_integer_sequence<int, 15 - K>{});
    a[K] = la;
    b[K] = lb;
    if constexpr (K < 15) step2<K + 1, NW>(a, b);
}

template <int V>
__global__ __launch_bounds__(64) void probe(const double* A, double* out, unsigned long long* cyc, int reps) {
    const int i = threadIdx.x & 63;
    double a0[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) a0[j] = (i < 16 && j <= i) ? A[i * 16 + j] : (i == j ? 1.0 : 0.0);
    double sink = 0.0;
    const unsigned long long t0 = stamp();
    for (int r = 0; r < reps; ++r) {
        double a[16], x[16], b[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) { a[j] = a0[j] + sink * 1e-300; b[j] = a[j]; x[j] = 0.0; }
        if constexpr (V == 0) step<0, true, 2, false>(a, x, i);
        if constexpr (V == 1) step<0, false, 2, false>(a, x, i);
        if constexpr (V == 2) step<0, true, 1, false>(a, x, i);
        if constexpr (V == 3) step<0, false, 1, false>(a, x, i);
        if constexpr (V == 4) step2<0, 2>(a, b);
        if constexpr (V == 5) step<0, true, 2, true>(a, x, i);
        if constexpr (V == 6) step<0, false, 2, true>(a, x, i);
        if constexpr (V == 7) bstep<0>(a, x, 1.0);
        if constexpr (V == 8) hstep<0>(a, x, i);
#pragma unroll
        for (int j = 0; j < 16; ++j) sink += a[j] + x[j] + b[j];
    }
    const unsigned long long t1 = stamp();
    out[i] = sink;
    if (i == 0) cyc[V] = t1 - t0;
}


// interference: wave 0 times the current factor (in-register, as above) while
// the other waves of a 512-thread workgroup run H until wave 0 is done:
// 0 idle (return), 1 fp64 MFMA chains, 2 LDS reads/writes, 3 fp64 VALU FMAs,
// 4 s_sleep; SIMD0ONLY: only wave 4 (wave 0's SIMD mate) runs H, others idle
typedef double v4d __attribute__((ext_vector_type(4)));
template <int H, bool SIMD0ONLY>
__global__ __launch_bounds__(512) void interf(const double* A, double* out, unsigned long long* cyc, int reps) {
    __shared__ double lds[64 * 65];
    __shared__ int done;
    const int wave = threadIdx.x >> 6, i = threadIdx.x & 63;
    if (threadIdx.x == 0) done = 0;
    for (int e = threadIdx.x; e < 64 * 65; e += 512) lds[e] = 1e-3 * e;
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
            step<0, true, 2, false>(a, x, i);
            sink += a[15] + x[15];
        }
        const unsigned long long t1 = stamp();
        __builtin_amdgcn_s_setprio(0);
        out[i] = sink;
        if (i == 0) cyc[0] = t1 - t0;
        __hip_atomic_store(&done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return;
    }
    if (H == 0 || (SIMD0ONLY && wave != 4)) return;
    v4d acc = {0, 0, 0, 0};
    double v = lds[i], w = 0.0;
    while (__hip_atomic_load(&done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
        for (int it = 0; it < 16; ++it) {
            if constexpr (H == 1) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, acc, 0, 0, 0);
            if constexpr (H == 2) { lds[(wave * 64 + i + it * 7) % (64 * 65)] = v; v = lds[(i * 65 + it) % (64 * 65)]; }
            if constexpr (H == 3) { w = fma(v, w, 1.0); v = fma(w, v, 0.5); }
            if constexpr (H == 4) __builtin_amdgcn_s_sleep(8);
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
    hipMalloc(&dA, 256 * 8); hipMalloc(&dout, 64 * 8); hipMalloc(&dc, 16 * 8);
    hipMemcpy(dA, A.data(), 256 * 8, hipMemcpyHostToDevice);
    const int reps = 2000;
    const char* names[] = {"current (x rows, 2 Newton, asm)", "no x rows", "x rows, 1 Newton", "no x rows, 1 Newton",
                           "two factors interleaved (no x)", "x rows, C-level update", "no x rows, C-level update",
                           "Bareiss chain (no L, no x)", "x rows, Halley rsq"};
    for (int pass = 0; pass < 2; ++pass) {
        probe<0><<<1, 64>>>(dA, dout, dc, reps); probe<1><<<1, 64>>>(dA, dout, dc, reps);
        probe<2><<<1, 64>>>(dA, dout, dc, reps); probe<3><<<1, 64>>>(dA, dout, dc, reps);
        probe<4><<<1, 64>>>(dA, dout, dc, reps); probe<5><<<1, 64>>>(dA, dout, dc, reps);
        probe<6><<<1, 64>>>(dA, dout, dc, reps); probe<7><<<1, 64>>>(dA, dout, dc, reps);
        probe<8><<<1, 64>>>(dA, dout, dc, reps);
        hipDeviceSynchronize();
    }
    unsigned long long c[16];
    hipMemcpy(c, dc, 16 * 8, hipMemcpyDeviceToHost);
    {
        const char* hn[] = {"idle", "mfma f64", "lds", "valu f64", "s_sleep"};
        unsigned long long cc;
        auto run = [&](auto kern, const char* what, const char* mode) {
            for (int pass = 0; pass < 2; ++pass) kern<<<1, 512>>>(dA, dout, dc, 500);
            hipDeviceSynchronize();
            hipMemcpy(&cc, dc, 8, hipMemcpyDeviceToHost);
            printf("in a 512-thread WG, helpers %-9s (%s): %8.0f cycles/factor\n", what, mode, (double)cc / 500);
        };
        run(interf<0, false>, hn[0], "all"); run(interf<1, false>, hn[1], "all"); run(interf<2, false>, hn[2], "all");
        run(interf<3, false>, hn[3], "all"); run(interf<4, false>, hn[4], "all");
        run(interf<1, true>, hn[1], "wave 4 only"); run(interf<2, true>, hn[2], "wave 4 only");
        run(interf<3, true>, hn[3], "wave 4 only");
    }
    for (int v = 0; v < 9; ++v)
        printf("%-36s %8.0f cycles/factor  %6.1f /pivot\n", names[v], (double)c[v] / reps, (double)c[v] / reps / 16);
    return 0;
}
