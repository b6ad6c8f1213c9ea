// Reduced-camera-system solve by block cyclic reduction (BCR).
//
// The RCS of a camera sequence is block-banded (half-bandwidth D camera
// blocks) plus a dense arrow for the shared intrinsics.  Grouping K = 10
// consecutive 6-dof camera blocks (K >= D) into 64x64 super-blocks makes the
// band block-tridiagonal; cyclic reduction then eliminates every other
// super-block in parallel, log2(N) levels deep, instead of walking 6000
// pivots one after another.  The arrow is handled by bordering: the band is
// solved for [rhs | arrow'] (1 + 4*nintr right-hand sides), then the small
// corner system, then y_band = y0 - Y_arrow x_corner.
//
// Mathematically the same direct solution ceres' SPARSE_SCHUR + EIGEN_SPARSE
// computes for the reduced camera system (BundleAdjuster.h:171-173).
//
// Dense 64x64 work is blocked in 16x16 tiles: each diagonal tile is factored
// and inverted inside one wavefront (no block barriers), everything else is
// fp64 MFMA (v_mfma_f64_16x16x4_f64) tile products.  A factored super-block
// keeps X = L^-1 explicitly, so every triangular solve is a product.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <type_traits>
#include <utility>

#include "ba_bcr.h"
#include "ba_cand.h"
#include "common.h"

// Inter-workgroup hand-offs in this file use the counter form of
// cdna_hip_programming.md Guideline 16: payloads stored and loaded with
// agent-scope relaxed atomics (sc1: written through / read past the CU's L1),
// drained with s_waitcnt vmcnt(0) (on gfx9 the vector memory counter also
// counts stores), then a relaxed agent-scope ticket or flag -- no release or
// acquire fence.  That is a property of the gfx950 ISA and its cache
// policy, not of the HIP memory model, so the device code refuses to build
// for any other target.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "counter-form hand-offs (sc1 payloads + vmcnt drain + relaxed ticket) are written for gfx950 only"
#endif

namespace sfm {
namespace {

constexpr int M = kBcrM;      // 64
constexpr int LD = M + 1;     // LDS row stride (bank spread)
constexpr int NT = 256;

// The published solve verdict (kScSolveFail): 0 ok, 1 numerical failure (a
// non-positive pivot: the LM loop's invalid step), kSolveWaitTimeout when a
// dataflow wait timed out (fail[1]: a workgroup was not resident, e.g. another
// context held the CUs; the host reports SFM_ERR_DEVICE instead of counting
// an invalid step).
__device__ __forceinline__ double solve_verdict(const double* fail) {
    const double t = __hip_atomic_load(fail + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return t != 0.0 ? kSolveWaitTimeout : __hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// after the verdict: the failure words start the next solve cleared (they
// are zeroed once at allocation; no pack launch clears them)
__device__ __forceinline__ void reset_verdict(const BcrArgs& b) {
    __hip_atomic_store(b.fail, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(b.fail + 1, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// rows of a super-block that can be nonzero in its W / z blocks (K cameras:
// 6K real rows, rounded up to the MFMA's k step of 4; K is 9 or 10): the
// products over block rows stop here (C4, K = 9: 56 of 64).  Written so the
// compiler sees 56 <= kM <= 64.
__device__ __forceinline__ int bcr_kM(const BcrArgs& b) { return b.K <= 9 ? 56 : b.K == 10 ? 60 : 64; }

__device__ __forceinline__ double clampd(double v, double lo, double hi) { return fmin(fmax(v, lo), hi); }

// Global-address-space agent-scope accesses for words handed between
// workgroups of one launch (sc1: written through / read past this CU's L1;
// cdna_hip_programming.md Guideline 16)
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) double gf64;
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store((gf64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __hip_atomic_load((gf64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

typedef double v4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 1/sqrt(d): the hardware estimate (v_rsq_f64, relative error below 2^-22)
// and one Newton step (relative error ~1e-13, well inside the solve's
// tolerance; a second step cost 4 of the pivot's ~33 instructions:
// tools/probe/diag16_variants.hip, profiles/r05/g_ab)
__device__ __forceinline__ double rsqrt_nr(double d) {
    const double y = __builtin_amdgcn_rsq(d);
    return fma(y, fma(-(0.5 * d * y), y, 0.5), y);
}

// One wave, one 16x16 output tile: acc += op(A)[ar.., k] op(B)[k, bc..] for
// k in [k0, k1) (k1 - k0 a multiple of 16).  op(A)[m][k] = TA ? A[k][m] : A[m][k],
// op(B)[k][n] = TB ? B[n][k] : B[k][n].  NEG negates the product.  The LDS
// operands of the next 16-wide k chunk are read while the current chunk's four
// MFMAs run, so a runtime-length product is not LDS-latency bound.
template <bool TA, bool TB, bool NEG, class PA = const double*, class PB = const double*>
__device__ __forceinline__ v4d tile_mm(v4d acc, PA A, int lda, int ar, PB B, int ldb, int bc, int k0, int k1) {
    const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4;
    double a[4], b[4];
    auto load = [&](int k, double (&av)[4], double (&bv)[4]) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int kj = k + 4 * j + kk;
            av[j] = TA ? A[kj * lda + ar + i] : A[(ar + i) * lda + kj];
            bv[j] = TB ? B[(bc + i) * ldb + kj] : B[kj * ldb + bc + i];
        }
    };
    load(k0, a, b);
    for (int k = k0; k < k1; k += 16) {
        double an[4], bn[4];
        const bool more = k + 16 < k1;
        if (more) load(k + 16, an, bn);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(NEG ? -a[j] : a[j], b[j], acc, 0, 0, 0);
        if (more) {
#pragma unroll
            for (int j = 0; j < 4; ++j) { a[j] = an[j]; b[j] = bn[j]; }
        }
    }
    return acc;
}
// Out-of-line tile products for the level kernel.  Its eight waves run
// different code at the same time, and with every product inlined the kernel
// was 61 KB of code: past the 64 KB instruction cache two CUs share, so the
// pivot wave's diagonal factor waited on instruction fetches.  Operands are
// typed by address space (LDS: ds_read; global: global_load), since a
// generic pointer through a call would become flat accesses.
typedef __attribute__((address_space(3))) const double lds_cd;
template <bool TA, bool TB, bool NEG>
__device__ __noinline__ v4d mm_ll(v4d acc, lds_cd* A, int lda, int ar, lds_cd* B, int ldb, int bc, int k0, int k1) {
    // k1 - k0 is 16, 32, 48 or 64: every chunk's reads first, then the MFMA
    // chain (the scheduler otherwise waits a full LDS latency per chunk)
    const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4;
    const int nc = (k1 - k0) >> 4;
    double a[16], b[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (c < nc) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int kj = k0 + 16 * c + 4 * j + kk;
                a[4 * c + j] = TA ? A[kj * lda + ar + i] : A[(ar + i) * lda + kj];
                b[4 * c + j] = TB ? B[(bc + i) * ldb + kj] : B[kj * ldb + bc + i];
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (c < nc) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(NEG ? -a[4 * c + j] : a[4 * c + j], b[4 * c + j], acc, 0, 0, 0);
        }
    }
    return acc;
}
// the same over block rows k in [0, kM), kM in {56, 60, 64}: a super-block's
// K real cameras fill 6K of its 64 rows and its W / z rows beyond them are
// zero, so the last 16-deep chunk multiplies only its first kM - 48 rows
// (C4, K = 9: 14 of 16 MFMAs); the branches are uniform and in the tail only
template <bool TA, bool TB, bool NEG>
__device__ __noinline__ v4d mm_ll_rows(v4d acc, lds_cd* A, int lda, int ar, lds_cd* B, int ldb, int bc, int kM) {
    const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4;
    // every operand read first (16 k steps, 64 VGPRs), then the MFMA chain
    double a[16], b[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int kj = 4 * q + kk;
        a[q] = TA ? A[kj * lda + ar + i] : A[(ar + i) * lda + kj];
        b[q] = TB ? B[(bc + i) * ldb + kj] : B[kj * ldb + bc + i];
    }
    // (without this the scheduler sinks each read next to its MFMA, which
    // then waits a full LDS latency every step)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 16; ++q)
        if (q < 14 || 4 * q < kM) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(NEG ? -a[q] : a[q], b[q], acc, 0, 0, 0);
    return acc;
}
// A 64 x 16 column block of a global matrix held in registers, in the
// operand order of tile_mm's k loop (v[4 c + j]: row 16 c + 4 j + kk, column
// i).  The level kernel's neighbour products (C_i, C_r, R_i updates) fetch
// their global operand this way at the start of a window, so the product
// runs at LDS speed instead of waiting one L2 latency per 16-deep k chunk.
struct GTile {
    double v[16];
    __device__ __forceinline__ void fetch(const double* p, int ld) {
        const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4;
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j) v[4 * c + j] = p[(16 * c + 4 * j + kk) * ld + i];
    }
};
// acc +/-= A[k][ar + m]' G[k][n], k = 0..kM-1 (A in LDS, transposed)
template <bool NEG, class PA>
__device__ __forceinline__ v4d mm_tr(v4d acc, PA A, int lda, int ar, const GTile& g, int kM) {
    const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4;
    double a[16];   // every LDS operand read first (mm_ll)
#pragma unroll
    for (int q = 0; q < 16; ++q) a[q] = A[(4 * q + kk) * lda + ar + i];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 16; ++q)
        if (q < 14 || 4 * q < kM)   // rows >= kM are zero (mm_ll_rows)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(NEG ? -a[q] : a[q], g.v[q], acc, 0, 0, 0);
    return acc;
}
// acc +/-= G[k][m]' B[k][bc + n], k = 0..kM-1 (B in LDS)
template <bool NEG, class PB>
__device__ __forceinline__ v4d mm_rt(v4d acc, const GTile& g, PB B, int ldb, int bc, int kM) {
    const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4;
    double bv[16];   // every LDS operand read first (mm_ll)
#pragma unroll
    for (int q = 0; q < 16; ++q) bv[q] = B[(4 * q + kk) * ldb + bc + i];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 16; ++q)
        if (q < 14 || 4 * q < kM)   // rows >= kM are zero (mm_ll_rows)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(NEG ? -g.v[q] : g.v[q], bv[q], acc, 0, 0, 0);
    return acc;
}
__device__ __forceinline__ lds_cd* L3(const double* p) { return (lds_cd*)p; }

__device__ __forceinline__ v4d tile_ld(const double* C, int ldc, int r0, int c0) {
    const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4;
    v4d v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = C[(r0 + kk + 4 * r) * ldc + c0 + i];
    return v;
}
__device__ __forceinline__ void tile_st(double* C, int ldc, int r0, int c0, v4d v) {
    const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) C[(r0 + kk + 4 * r) * ldc + c0 + i] = v[r];
}
__device__ __forceinline__ v4d zero4() { return v4d{0.0, 0.0, 0.0, 0.0}; }

// global [R][ld_src] -> LDS [R][ld_dst], first NC columns: every thread
// issues all its 16-byte loads before the first LDS store
template <int NC, int R = M, int TH = NT>
__device__ __forceinline__ void load_tile(double* dst, int ld_dst, const double* __restrict__ src, int ld_src) {
    constexpr int n2 = R * NC / 2, per = (n2 + TH - 1) / TH;
    double2 v[per];
#pragma unroll
    for (int q = 0; q < per; ++q) {
        const int e = threadIdx.x + q * TH;
        if (e < n2) v[q] = *reinterpret_cast<const double2*>(src + (e / (NC / 2)) * ld_src + 2 * (e % (NC / 2)));
    }
#pragma unroll
    for (int q = 0; q < per; ++q) {
        const int e = threadIdx.x + q * TH;
        if (e < n2) {
            double* d = dst + (e / (NC / 2)) * ld_dst + 2 * (e % (NC / 2));
            d[0] = v[q].x;
            d[1] = v[q].y;
        }
    }
}
// a tile's global -> LDS copy split in two: fetch (every 16-byte load of the
// thread issued) and put (LDS stores), so several tiles' loads can be in flight
// together -- one memory latency for all of them instead of one per tile
template <int NC, int R = M, int TH = NT>
struct TileFetch {
    static constexpr int n2 = R * NC / 2, per = (n2 + TH - 1) / TH;
    double2 v[per];
    __device__ __forceinline__ void fetch(const double* __restrict__ src, int ld_src) {
#pragma unroll
        for (int q = 0; q < per; ++q) {
            const int e = threadIdx.x + q * TH;
            if (e < n2) v[q] = *reinterpret_cast<const double2*>(src + (e / (NC / 2)) * ld_src + 2 * (e % (NC / 2)));
        }
    }
    __device__ __forceinline__ void put(double* dst, int ld_dst) const {
#pragma unroll
        for (int q = 0; q < per; ++q) {
            const int e = threadIdx.x + q * TH;
            if (e < n2) {
                double* d = dst + (e / (NC / 2)) * ld_dst + 2 * (e % (NC / 2));
                d[0] = v[q].x;
                d[1] = v[q].y;
            }
        }
    }
};
// two 64x64 global tiles -> LDS [64][LD], every load of both in flight before
// the first LDS store (one memory latency instead of two)
__device__ __forceinline__ void load_tiles2(double* d1, const double* __restrict__ s1, double* d2,
                                            const double* __restrict__ s2, int ld_src) {
    constexpr int n2 = M * M / 2, per = n2 / NT;
    double2 v[2 * per];
#pragma unroll
    for (int q = 0; q < per; ++q) {
        const int e = threadIdx.x + q * NT, r = e / (M / 2), c = 2 * (e % (M / 2));
        v[q] = *reinterpret_cast<const double2*>(s1 + r * ld_src + c);
        v[per + q] = *reinterpret_cast<const double2*>(s2 + r * ld_src + c);
    }
#pragma unroll
    for (int q = 0; q < per; ++q) {
        const int e = threadIdx.x + q * NT, r = e / (M / 2), c = 2 * (e % (M / 2));
        d1[r * LD + c] = v[q].x;
        d1[r * LD + c + 1] = v[q].y;
        d2[r * LD + c] = v[per + q].x;
        d2[r * LD + c + 1] = v[per + q].y;
    }
}
// up to four 64x64 global tiles -> LDS [64][LD] (tiles t < n), every load in
// flight before the first LDS store (one memory latency for all of them)
__device__ __forceinline__ void load_tiles4(int n, double* d0, const double* s0, double* d1, const double* s1,
                                            double* d2, const double* s2, double* d3, const double* s3, int ld_src) {
    constexpr int n2 = M * M / 2, per = n2 / NT;
    double* const dd[4] = {d0, d1, d2, d3};
    const double* const ss[4] = {s0, s1, s2, s3};
    double2 v[4][per];
#pragma unroll
    for (int t = 0; t < 4; ++t)
        if (t < n) {
#pragma unroll
            for (int q = 0; q < per; ++q) {
                const int e = threadIdx.x + q * NT, r = e / (M / 2), c = 2 * (e % (M / 2));
                v[t][q] = *reinterpret_cast<const double2*>(ss[t] + r * ld_src + c);
            }
        }
#pragma unroll
    for (int t = 0; t < 4; ++t)
        if (t < n) {
#pragma unroll
            for (int q = 0; q < per; ++q) {
                const int e = threadIdx.x + q * NT, r = e / (M / 2), c = 2 * (e % (M / 2));
                dd[t][r * LD + c] = v[t][q].x;
                dd[t][r * LD + c + 1] = v[t][q].y;
            }
        }
}
template <int TH = NT>
__device__ __forceinline__ void load_rows(double* dst, int ld_dst, const double* src, int ld_src, int nc) {
    if (nc == 64) load_tile<64, M, TH>(dst, ld_dst, src, ld_src);
    else if (nc == 32) load_tile<32, M, TH>(dst, ld_dst, src, ld_src);
    else load_tile<16, M, TH>(dst, ld_dst, src, ld_src);
}

// value of v in lane l of this lane's 16-lane row (DPP row_newbcast, 64-bit);
// l must fold to a constant
__device__ __forceinline__ double row_bcast(double v, int l) {
#define SFM_BC(n) case n: return __builtin_amdgcn_mov_dpp(v, 0x150 + n, 0xf, 0xf, true);
    switch (l) {
        SFM_BC(0) SFM_BC(1) SFM_BC(2) SFM_BC(3) SFM_BC(4) SFM_BC(5) SFM_BC(6) SFM_BC(7)
        SFM_BC(8) SFM_BC(9) SFM_BC(10) SFM_BC(11) SFM_BC(12) SFM_BC(13) SFM_BC(14)
        default: return __builtin_amdgcn_mov_dpp(v, 0x15f, 0xf, 0xf, true);
    }
#undef SFM_BC
}

// acc += (src of lane l of this lane's 16-lane row) * mul, one v_fmac_f64 with
// a DPP row_newbcast source.  The compiler does not see inside the asm, so the
// DPP read-after-VALU-write hazard (2 wait states) is covered by NOP = true on
// the first FMA of each group; tests/test_bcr_asm.py checks the schedule.
#define SFM_FMAC_BC(n)                                                                                 \
    case n:                                                                                            \
        if (NOP && NEG)                                                                                \
            asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:" #n " row_mask:0xf bank_mask:0xf" \
                         : "+v"(acc) : "v"(src), "v"(mul));                                            \
        else if (NOP)                                                                                  \
            asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:" #n " row_mask:0xf bank_mask:0xf" \
                         : "+v"(acc) : "v"(src), "v"(mul));                                            \
        else if (NEG)                                                                                  \
            asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:" #n " row_mask:0xf bank_mask:0xf"  \
                         : "+v"(acc) : "v"(src), "v"(mul));                                            \
        else                                                                                           \
            asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #n " row_mask:0xf bank_mask:0xf"   \
                         : "+v"(acc) : "v"(src), "v"(mul));                                            \
        break;
template <bool NOP, bool NEG = false>
__device__ __forceinline__ void fmac_bc(double& acc, double src, double mul, int l) {
    switch (l) {
        SFM_FMAC_BC(0) SFM_FMAC_BC(1) SFM_FMAC_BC(2) SFM_FMAC_BC(3) SFM_FMAC_BC(4) SFM_FMAC_BC(5)
        SFM_FMAC_BC(6) SFM_FMAC_BC(7) SFM_FMAC_BC(8) SFM_FMAC_BC(9) SFM_FMAC_BC(10) SFM_FMAC_BC(11)
        SFM_FMAC_BC(12) SFM_FMAC_BC(13) SFM_FMAC_BC(14) SFM_FMAC_BC(15)
        default: break;
    }
}
#undef SFM_FMAC_BC

// Wave-local factor + inverse of one 16x16 diagonal tile: lane i < 16 owns
// row i of A in registers and column i of X = L^-1.  Step k broadcasts the
// unscaled column k of every row across the 16 lanes with DPP row_newbcast
// folded into the FMAs (no LDS, no scalar round trip) and applies
// a_ij -= (a_ik / d_k) a_jk.  Row k of X (x_k = (e_k - sum_p L_kp x_p) / L_kk)
// is computed as soon as row k of L is final.  Single-wave issue bound:
// about 30 fp64 instructions per pivot.
// X gets L^-1 (upper zeroed); the tile of A is left as it was loaded.
// step K of diag16, expanded at compile time (an inline-asm body defeats the
// loop unroller, and every broadcast lane must be an immediate)
template <int K, int... J>
__device__ __forceinline__ void diag16_update(double (&a)[16], double nt, std::integer_sequence<int, J...>) {
    (fmac_bc<J == 0>(a[K + 1 + J], a[K], nt, K + 1 + J), ...);
}
template <int K, bool NEG, int... P>
__device__ __forceinline__ void diag16_xrow(const double (&a)[16], const double (&x)[16], double& u0, double& u1,
                                            std::integer_sequence<int, P...>) {
    ((P & 1 ? fmac_bc<false, NEG>(u1, a[P], x[P], K) : fmac_bc<P == 0, NEG>(u0, a[P], x[P], K)), ...);
}
// The wave is VALU-issue bound here (one wave, fp64: ~8 cycles per
// instruction), so each pivot is kept to few instructions: no select for the
// new column (lane K's a_KK is d, so lk = a_iK rinv is L_KK on lane K, L_iK
// below it, and only the never-read upper triangle above) and no per-pivot
// definiteness test (a pivot d <= 0 or NaN leaves a non-positive or NaN L_KK,
// checked once at the end).
template <int K, int NP>
__device__ __forceinline__ void diag16_step(double (&a)[16], double (&x)[16], int i) {
    const double d = row_bcast(a[K], K);
    const double rinv = rsqrt_nr(d);
    const double lk = a[K] * rinv;       // L_iK (i >= K)
    const double nt = -(lk * rinv);      // -a_iK / d_K
    diag16_update<K>(a, nt, std::make_integer_sequence<int, 15 - K>{});
    a[K] = lk;
    // row K of L is final: lane c gets x_K = (delta_Kc - sum_p L_Kp x_p) / L_KK;
    // x holds the identity's column until row K is formed, so the sum starts
    // from delta_Kc and subtracts (a negated DPP source: no select per pivot)
    (void)i;
    double u0 = x[K], u1 = 0.0;
    diag16_xrow<K, true>(a, x, u0, u1, std::make_integer_sequence<int, K>{});
    x[K] = (u0 + u1) * rinv;
    if constexpr (K + 1 < NP) diag16_step<K + 1, NP>(a, x, i);
}

// NP: pivots taken.  Rows NP..15 are a super-block's identity padding (the
// 6K real rows of a block of K cameras end inside its last diagonal tile:
// bcr_pack_kernel writes 1 on their diagonal and 0 elsewhere, and every
// update leaves them so, since their rows and columns of each C, W and z are
// zero): their L and X rows are the identity, so their pivots are skipped
// (K = 9: 10 of the 64 pivots of a super-block).
template <int NP = 16>
__device__ __forceinline__ void diag16_body(double* A, double* X, double* bad, double* col) {
    (void)col;
    // the critical path of the factorisation: ahead of the co-resident helper
    // waves (trailing tiles, background products) in VALU issue arbitration
    __builtin_amdgcn_s_setprio(2);
    const int lane = threadIdx.x & 63, i = lane;
    const bool act = lane < 16;
    // every caller's A and X are LDS tiles: address them as such (ds_* instead
    // of flat accesses, which wait on both counters), and load every row
    // unconditionally (lane i & 15), masking after, instead of 16 branches
    typedef __attribute__((address_space(3))) double lds_f64;
    lds_f64* const Al = (lds_f64*)A;
    lds_f64* const Xl = (lds_f64*)X;
    double a[16], x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = Al[(i & 15) * LD + j];
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = (act && j <= i) ? a[j] : 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = j == i ? 1.0 : 0.0;
    diag16_step<0, NP>(a, x, i);
    // (rows NP..15, the identity padding: x keeps the identity it started from, a keeps it too)
    double lii = 1.0;   // this lane's L_ii (a[i], extracted without dynamic indexing)
#pragma unroll
    for (int j = 0; j < 16; ++j) lii = j == i ? a[j] : lii;
    if (__ballot(act && !(lii > 0.0)) != 0 && lane == 0) bad[0] = 1.0;
    // only X = L^-1 goes back: nothing reads a factored diagonal tile of L
    // (panels are A X', the inverse's off-diagonal tiles sums of L_nm X_mj
    // with m < n), so its 16 stores are off the pivot wave's critical path
    if (act) {
#pragma unroll
        for (int m = 0; m < 16; ++m) Xl[m * LD + i] = x[m];
    }
    __builtin_amdgcn_s_setprio(0);
}

// called (BCR level / top kernels: inlined there it costs the helper waves'
// registers, 47 spilled VGPRs) or inlined (the dense kernels: 6 % faster
// factor, no spills)
template <int NP = 16>
__device__ __noinline__ void diag16(double* A, double* X, double* bad, double* col) { diag16_body<NP>(A, X, bad, col); }
// the last diagonal tile of a super-block: np3 = 6 K - 48 real pivots
__device__ __forceinline__ void diag16_last(int np3, double* A, double* X, double* bad, double* col) {
    if (np3 == 6) diag16<6>(A, X, bad, col);
    else if (np3 == 12) diag16<12>(A, X, bad, col);
    else diag16<16>(A, X, bad, col);
}

// Blocked Cholesky A = L L' of a 64x64 LDS tile and X = L^-1 (X zeroed by
// the caller).  All 256 threads; ends synchronised.
//
// Look-ahead schedule: the critical path is the four wave-local diagonal
// factors (VALU-issue bound) joined by one tile product each way:
//   P(k)   panels L_ik = A_ik X_kk' (i > k) and X_kj = -X_kk T_kj (j < k):
//          at most three tiles, one MFMA product each, waves 0..2
//   D(k+1) wave 0: A_{k+1,k+1} -= L_{k+1,k} L_{k+1,k}', then diag16(k+1);
//          waves 1..3 meanwhile: the other trailing tiles of step k and the
//          partial inverse rows T_{k+1,j} = sum_{m=j..k} L_{k+1,m} X_mj
// pre0 / preN: work that must precede the factorisation but only the first
// diagonal tile has to wait for: wave 0 runs pre0 (the update of A_00) and
// goes straight on to diag16(0); the other waves run preN (the remaining
// update tiles and anything else due before the first barrier) meanwhile.
// bg(k): background work of the helper waves in the window of diag16(k+1)
// (k = 0..2), after their trailing tiles (they idle there otherwise).
struct NoPre {
    __device__ void operator()() const {}
};
struct NoBg {
    __device__ void operator()(int) const {}
};
// np3: real pivots of the last diagonal tile (16: no padding; the BCR
// super-blocks' 6 K - 48)
template <int NW = NT / 64, class Pre0 = NoPre, class PreN = NoPre, class Bg = NoBg, bool INL = false>
__device__ __forceinline__ void chol_inv64(double* A, double* X, double* bad, double* col,
                           unsigned long long* st = nullptr, Pre0 pre0 = Pre0(), PreN preN = PreN(),
                           Bg bg = Bg(), int np3 = 16) {
    const int wave = threadIdx.x >> 6;
    unsigned long long t0 = 0, td = 0, ta = 0, tq = 0, tb = 0, tw = 0;
    // diagnostic (st): per window k (diag16(k) and the helpers' work beside
    // it) the pivot wave's and the slowest helper's cycles, LDS maxima in the
    // (otherwise unused) diag16 column scratch
    unsigned long long* wmax = reinterpret_cast<unsigned long long*>(col);
    if (st) {
        if (threadIdx.x < 8) wmax[threadIdx.x] = 0;
        __syncthreads();
        t0 = stamp();
    }
    auto wend = [&](int k) {   // this wave's window k is done
        if (st && (threadIdx.x & 63) == 0)
            atomicMax(wmax + (wave == 0 ? 4 : 0) + k, stamp() - tw);
    };
    tw = t0;
    if (wave == 0) {
        pre0();
        wave_sync();
        if (st) tb = stamp();
        if constexpr (INL) diag16_body(A, X, bad, col);
        else diag16(A, X, bad, col);
        if (st) {
            const unsigned long long te = stamp();
            td += te - t0;
            tq += te - tb;
        }
    } else {
        preN();
    }
    wend(0);
    __syncthreads();
    for (int k = 0;; ++k) {
        // ---- P(k): 3 - k panels, then k inverse tiles ----------------------
        if (wave < 3) {
            if (wave < 3 - k) {
                const int i = k + 1 + wave;
                tile_st(A, LD, 16 * i, 16 * k,
                        tile_mm<false, true, false>(zero4(), A, LD, 16 * i, X, LD, 16 * k, 16 * k, 16 * k + 16));
            } else {
                const int j = wave - (3 - k);   // T_kj sits in X tile (k, j)
                tile_st(X, LD, 16 * k, 16 * j,
                        tile_mm<false, false, true>(zero4(), X, LD, 16 * k, X, LD, 16 * j, 16 * k, 16 * k + 16));
            }
        }
        __syncthreads();
        if (k == 3) break;
        // ---- D(k+1) ---------------------------------------------------------
        const int n = k + 1;
        if (st) tw = stamp();
        if (wave == 0) {
            if (st) ta = stamp();
            v4d acc = tile_ld(A, LD, 16 * n, 16 * n);
            acc = tile_mm<false, true, true>(acc, A, LD, 16 * n, A, LD, 16 * n, 16 * k, 16 * k + 16);
            tile_st(A, LD, 16 * n, 16 * n, acc);
            wave_sync();
            if (st) tb = stamp();
            if constexpr (INL) diag16_body(A + 16 * n * (LD + 1), X + 16 * n * (LD + 1), bad, col);
            else if (n == 3) diag16_last(np3, A + 16 * n * (LD + 1), X + 16 * n * (LD + 1), bad, col);
            else diag16(A + 16 * n * (LD + 1), X + 16 * n * (LD + 1), bad, col);
            if (st) {
                const unsigned long long te = stamp();
                td += te - ta;
                tq += te - tb;
            }
        } else {
            // items: trailing tiles (i, j), n <= j <= i < 4, (i, j) != (n, n);
            // then T_nj, j < n
            int t = 0;
            for (int i = n; i < 4; ++i)
                for (int j = n; j <= i; ++j) {
                    if (i == n && j == n) continue;
                    if (t++ % (NW - 1) == wave - 1) {
                        v4d acc = tile_ld(A, LD, 16 * i, 16 * j);
                        acc = tile_mm<false, true, true>(acc, A, LD, 16 * i, A, LD, 16 * j, 16 * k, 16 * k + 16);
                        tile_st(A, LD, 16 * i, 16 * j, acc);
                    }
                }
            for (int j = 0; j < n; ++j)
                if (t++ % (NW - 1) == wave - 1)   // X is lower triangular: m runs j..n-1
                    tile_st(X, LD, 16 * n, 16 * j,
                            tile_mm<false, false, false>(zero4(), A, LD, 16 * n, X, LD, 16 * j, 16 * j, 16 * n));
            bg(k);
        }
        wend(n);
        __syncthreads();
    }
    if (st && threadIdx.x == 0) {
        atomicAdd(st + 0, td);
        atomicAdd(st + 1, stamp() - t0);
        atomicAdd(st + 7, tq);
        for (int q = 0; q < 8; ++q) atomicAdd(st + 8 + q, wmax[q]);
    }
}

// ---- pack: band (6x6 blocks) -> 64x64 super-blocks, D^2 added, identity pad --
// Element (r, c) of super-block I's A, C (block (I, I-1)) and R, gathered from
// the reduced band: every load is issued unconditionally from a clamped
// address and the value selected after, so a caller's unrolled loop keeps all
// its loads in flight.  The first level kernel gathers its blocks this way
// (bcr_pack_kernel remains for a band of one super-block).
struct PackIdx {
    int c0, nreal;
    __device__ PackIdx(const BcrArgs& b, const DevProblem& P, int I)
        : c0(I * b.K), nreal(min(b.K, P.ncam - I * b.K) * 6) {}
};
__device__ __forceinline__ double pack_a(const BcrArgs& b, const DevProblem& P, double radius, int I, int r, int c) {
    const PackIdx x(b, P, I);
    const int Dp = P.D + 1;
    const bool real = r < x.nreal && c < x.nreal;
    const int ci = x.c0 + r / 6, cj = x.c0 + c / 6;
    const int hi = max(ci, cj), lo = min(ci, cj), d = hi - lo;
    const bool inband = real && d <= P.D;
    // A: block (ci, cj) with cj in this super-block, cj <= ci (lower), mirror upper
    const int rr = ci >= cj ? r % 6 : c % 6, cc = ci >= cj ? c % 6 : r % 6;
    const double v = P.Sband[inband ? ((size_t)hi * Dp + d) * 36 + rr * 6 + cc : 0];
    const double cn = P.cnF[real ? 6LL * ci + r % 6 : 0];
    double a = inband ? v : 0.0;
    if (real && r == c) {
        const double lm = sqrt(clampd(cn, P.min_diag, P.max_diag) / radius);
        a += lm * lm;
    }
    return r >= x.nreal && r == c ? 1.0 : a;   // padding: identity
}
__device__ __forceinline__ double pack_c(const BcrArgs& b, const DevProblem& P, int I, int r, int c, bool on = true) {
    // block (ci, cj) with cj in the previous super-block (always full);
    // on = false: 0 (the load still issued, from a clamped address: no branch)
    const PackIdx x(b, P, I);
    const int Dp = P.D + 1;
    const int ci = x.c0 + r / 6, cj = x.c0 - b.K + c / 6, d = ci - cj;
    const bool ok = on && I > 0 && r < x.nreal && c / 6 < b.K && d >= 1 && d <= P.D;
    const double v = P.Sband[ok ? ((size_t)ci * Dp + d) * 36 + (r % 6) * 6 + c % 6 : 0];
    return ok ? v : 0.0;
}
// R: column 0 = rhs, columns 1 + iw k + a = arrow (intr k, row a) transposed
__device__ __forceinline__ double pack_r(const BcrArgs& b, const DevProblem& P, int I, int r, int c, bool on = true) {
    const PackIdx x(b, P, I);
    const int ci = x.c0 + r / 6;
    const bool real = on && r < x.nreal;
    const bool rhs = real && c == 0, arrow = real && c > 0 && c - 1 < P.iw * P.nintr;
    const int k = (c - 1) / P.iw, a = (c - 1) % P.iw;
    const double vr = P.rhs[rhs ? 6LL * ci + r % 6 : 0];
    const double va = P.Sarrow[arrow ? ((size_t)k * P.ncam + ci) * 6 * P.iw + a * 6 + r % 6 : 0];
    return rhs ? vr : arrow ? va : 0.0;
}
// The first level kernel's gathers: a thread's column c of super-block I is
// fixed, so its column terms -- and the one LM damping term its column can
// need (the diagonal element (c, c)) -- are formed once; rows vary per
// element.  Same values as pack_a (the damping is added to the band value in
// one rounding, as there).
struct BandCol {
    int c0, nreal, Dp, cj, cm;
    bool creal;
    double dmp;   // lm^2 of column c (0 for a padding column)
    __device__ BandCol(const BcrArgs& b, const DevProblem& P, double radius, int I, int c) {
        c0 = I * b.K;
        nreal = min(b.K, P.ncam - c0) * 6;
        Dp = P.D + 1;
        cj = c0 + c / 6;
        cm = c % 6;
        creal = c < nreal;
        const double cn = P.cnF[creal ? 6 * cj + cm : 0];
        const double lm = sqrt(clampd(cn, P.min_diag, P.max_diag) / radius);
        dmp = creal ? lm * lm : 0.0;
    }
    // element (r, c) of A
    __device__ __forceinline__ double a(const DevProblem& P, int r, int c) const {
        const int ci = c0 + r / 6, rm = r % 6;
        const bool real = r < nreal && creal;
        const int d = ci >= cj ? ci - cj : cj - ci;
        const bool inband = real && d <= P.D;
        const int idx = ci >= cj ? ((ci * Dp + d) * 36 + rm * 6 + cm) : ((cj * Dp + d) * 36 + cm * 6 + rm);
        const double v = P.Sband[inband ? idx : 0];
        double x = inband ? v : 0.0;
        x = (real && r == c) ? x + dmp : x;
        return r >= nreal && r == c ? 1.0 : x;   // padding: identity
    }
};
// rows [r0, r0 + 16) of super-block I's A and R, gathered to global memory
// (the first level kernel, for the even blocks beside its odd ones)
template <int TH>
__device__ __forceinline__ void pack_rows(const BcrArgs& b, const DevProblem& P, double radius, int I, int r0, int t) {
    double* A = b.A + (size_t)I * M * M + (size_t)r0 * M;
    double* R = b.R + (size_t)I * M * b.nrhs + (size_t)r0 * b.nrhs;
    static_assert(TH % M == 0, "a thread's column is fixed");
    constexpr int NA = 16 * M / TH;
    const BandCol col(b, P, radius, I, t % M);
    double va[NA];
#pragma unroll
    for (int q = 0; q < NA; ++q) {
        const int e = t + q * TH;
        va[q] = col.a(P, r0 + e / M, e % M);
    }
    static_assert(16 * 32 <= TH, "one R element per thread at most (nrhs <= 32)");
    const bool hasr = t < 16 * b.nrhs;
    const double vr = pack_r(b, P, I, r0 + t / b.nrhs, t % b.nrhs, hasr);
#pragma unroll
    for (int q = 0; q < NA; ++q) A[t + q * TH] = va[q];
    if (hasr) R[t] = vr;
}

// One workgroup per 4 rows of a super-block (N * 16 workgroups).
__global__ void bcr_pack_kernel(BcrArgs b, DevProblem P, double radius) {
    const int I = blockIdx.x >> 4, rg = blockIdx.x & 15;
    double* A = b.A + (size_t)I * M * M;
    double* Cm = b.C + (size_t)I * M * M;
    double* R = b.R + (size_t)I * M * b.nrhs;
    {
        const int e = 4 * rg * M + threadIdx.x;   // NT = 4 rows x 64 columns
        const int r = e / M, c = e % M;
        A[e] = pack_a(b, P, radius, I, r, c);
        Cm[e] = pack_c(b, P, I, r, c);
    }
    for (int e = 4 * rg * b.nrhs + threadIdx.x; e < 4 * (rg + 1) * b.nrhs; e += NT)
        R[e] = pack_r(b, P, I, e / b.nrhs, e % b.nrhs);
}

// ---- update of one 16-row tile w of an even block j after eliminating its odd
// neighbours at stride s (they hold Wl = L^-1 C, Wr = L^-1 C_r', z = L^-1 R):
// A_j -= Wr_{j-s}' Wr_{j-s} + Wl_{j+s}' Wl_{j+s};  R_j -= Wr' z + Wl' z.
// (The new coupling C_j is not formed: every odd block after the first level
// forms its C_i and C_r from the neighbours' W blocks itself.)  Wave v: tile (w, v).
template <int TH>
__device__ void update_tile_rows(const BcrArgs& b, int s, int j, int w, double* sm) {
    const int kM = bcr_kM(b);
    const int ldr = b.nrhs + 1;
    double* Wa = sm;               // Wr_{j-s}
    double* Wb = Wa + M * LD;      // Wl_{j+s}
    double* Za = Wb + M * LD;      // z_{j-s}
    double* Zb = Za + M * ldr;     // z_{j+s}
    // waves 0..3: A tile (w, v); waves 4..7: R and C tiles (w, v - 4)
    const int il = j - s, ir = j + s, wv = threadIdx.x >> 6, v = wv & 3;
    const bool hl = il >= 0, hr = ir < b.N;
    // every tile's loads in flight together (nrhs is 16 or 32: bcr_supported)
    auto loads = [&](auto ncz) {
        constexpr int NCZ = decltype(ncz)::value;
        TileFetch<64, M, TH> fwa, fwb;
        TileFetch<NCZ, M, TH> fza, fzb;
        if (hl) {
            fwa.fetch(b.Wr + (size_t)il * M * M, M);
            fza.fetch(b.Z + (size_t)il * M * b.nrhs, b.nrhs);
        }
        if (hr) {
            fwb.fetch(b.Wl + (size_t)ir * M * M, M);
            fzb.fetch(b.Z + (size_t)ir * M * b.nrhs, b.nrhs);
        }
        if (hl) {
            fwa.put(Wa, LD);
            fza.put(Za, ldr);
        }
        if (hr) {
            fwb.put(Wb, LD);
            fzb.put(Zb, ldr);
        }
    };
    if (b.nrhs == 16) loads(std::integral_constant<int, 16>{});
    else loads(std::integral_constant<int, 32>{});
    __syncthreads();
    double* Aj = b.A + (size_t)j * M * M;
    if (wv < 4) {
        v4d acc = tile_ld(Aj, M, 16 * w, 16 * v);
        if (hl) acc = mm_ll_rows<true, false, true>(acc, L3(Wa), LD, 16 * w, L3(Wa), LD, 16 * v, kM);
        if (hr) acc = mm_ll_rows<true, false, true>(acc, L3(Wb), LD, 16 * w, L3(Wb), LD, 16 * v, kM);
        tile_st(Aj, M, 16 * w, 16 * v, acc);
        return;
    }
    if (16 * v < b.nrhs) {
        double* Rj = b.R + (size_t)j * M * b.nrhs;
        v4d acc = tile_ld(Rj, b.nrhs, 16 * w, 16 * v);
        if (hl) acc = mm_ll_rows<true, false, true>(acc, L3(Wa), LD, 16 * w, L3(Za), ldr, 16 * v, kM);
        if (hr) acc = mm_ll_rows<true, false, true>(acc, L3(Wb), LD, 16 * w, L3(Zb), ldr, 16 * v, kM);
        tile_st(Rj, b.nrhs, 16 * w, 16 * v, acc);
    }
}

// ---- one cyclic-reduction level at stride s, one launch --------------------------
// Workgroups (item, w), w = 16-column / 16-row tile:
//   odd block i (items < n_odd): bring A_i, column tile w of C_i (block (i, i-s)),
//     row tile w of C_r (block (r, i), r = i+s) and column tile w of R_i up to
//     date with the previous level (stride s/2) in LDS -- each of the block's 4
//     workgroups does this redundantly -- factor A_i = L L', X = L^-1 (stored by
//     w = 0 for the back substitution), and store column tile w of
//     Wl = X C_i, Wr = X C_r', z = X R_i.
//   even block j (items >= n_odd, s > 1): update(s/2) of its row tile w, stored.
// At s = 1 the odd blocks gather their inputs straight from the reduced band
// (pack_a / pack_c / pack_r) and pack the even blocks' A and R rows for the
// later levels.
constexpr int NTL = 512, NWL = NTL / 64;   // level kernel: 8 waves

__device__ __forceinline__ void bcr_corner_body(const BcrArgs& b, const DevProblem& P, double radius, int I,
                                                bool z_fresh, bool part_done = false, unsigned tag = 0,
                                                const double* own = nullptr);
__device__ __forceinline__ void put_y(unsigned long long* g, int row, double v, unsigned epoch);
// block 0's corner partial (nrhs = 16: q00 only) into LDS, the part layout
// (the fused top: workgroup 0 keeps it and solves the corner itself)
__device__ __forceinline__ void corner_put_lds(const DevProblem& P, const v4d& q00, double* dst) {
    constexpr int kQ = 17;
    const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4, na = P.iw * P.nintr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int ga = kk + 4 * r, gc = i;
        if (ga >= 1 && ga <= na && gc <= na) dst[(ga - 1) * kQ + gc] = q00[r];
    }
}
// block I's corner partial (rows 1..na, columns 0..na of z_I' z_I) from this
// wave's MFMA results q00 (and, nrhs = 32, q10 / q11), stored write-through
__device__ __forceinline__ void corner_put(const BcrArgs& b, const DevProblem& P, int I, const v4d& q00,
                                           const v4d& q10, const v4d& q11, int ntc) {
    constexpr int kQ = 17;   // part row stride: columns 0..16
    const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4, na = P.iw * P.nintr;
    double* out = b.part + (size_t)I * 512;
    auto put = [&](const v4d& q, int r0, int c0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int ga = r0 + kk + 4 * r, gc = c0 + i;
            if (ga >= 1 && ga <= na && gc <= na) st_sc1(out + (ga - 1) * kQ + gc, q[r]);
        }
    };
    put(q00, 0, 0);
    if (ntc > 1) {
        put(q10, 16, 0);
        put(q11, 16, 16);
    }
}

// TOP (round 5): the root, super-block 0, as a level item with only its right
// neighbour sp = s / 2 (eliminated by the last level): workgroups 0..3 (w)
// factor A_0 - Wl_sp' Wl_sp with the level schedule and store row tile w of
// X_0 and column tile w of z_0 = X_0 (R_0 - Wl_sp' z_sp) -- no C_i / C_r
// outputs.  Fused launch (grid > 4): workgroups 4.. add the corner partials
// of blocks 1..N-1 meanwhile, and workgroup 0 adds block 0's after its z_0
// (bcr_corner_body; nrhs = 16 only, so that z_0 is one workgroup's).  The
// top used to be one workgroup with the barrier-phased chol_inv64.
template <bool TOP>
__global__ __launch_bounds__(NTL) void bcr_level_kernel(BcrArgs b, DevProblem P, double radius, int s, int n_odd,
                                                        unsigned epoch) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    int item, w;
    if constexpr (TOP) {
        if ((int)blockIdx.x >= 4) {
            bcr_corner_body(b, P, radius, (int)blockIdx.x - 3, false, false, epoch);
            return;
        }
        item = 0;
        w = blockIdx.x;
    } else {
        // XCD-aware: workgroup b runs on XCD b % 8, so the four workgroups (w) of
        // one item are b = x + 8 (4 j + w): the same XCD, whose L2 then serves the
        // block's A and neighbour W tiles once for all four
        const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;
        item = xcd + 8 * (q >> 2);
        w = q & 3;
    }
    const int sp = s >> 1;
    if (!TOP && item >= n_odd) {
        const int j = 2 * s * (item - n_odd);
        if (sp > 0 && j < b.N) update_tile_rows<NTL>(b, sp, j, w, sm);
        return;
    }
    const int i = TOP ? 0 : s + 2 * s * item;
    if (i >= b.N) return;
    const int r = i + s, wave = threadIdx.x >> 6;
    const bool hr = !TOP && r < b.N, hz = 16 * w < b.nrhs;
    const int np3 = 6 * b.K - 48;   // real pivots of the last diagonal tile
    const int kM = bcr_kM(b);
    constexpr int L16 = 17;
    double* A = sm;                 // [64][LD]
    double* X = A + M * LD;         // [64][LD]
    double* Wa_l = X + M * LD;      // [64][64] Wr_{i-sp}
    double* Wb_l = Wa_l + M * M;    // [64][64] Wl_{i+sp}
    double* Cc = Wb_l + M * M;      // [64][17] column tile w of C_i
    double* Cr = Cc + M * L16;      // [16][LD] row tile w of C_r
    double* Rc = Cr + 16 * LD;      // [64][17] column tile w of R_i
    double* bad = Rc + M * L16;
    double* col = bad + 2;          // [16] diag16 column scratch; stamp maxima (diagnostic)
    unsigned* pdone = reinterpret_cast<unsigned*>(col + 16);   // [4] P(k) items done (window hand-off)
    unsigned long long* st = (b.stamps && w == 0 && !TOP) ? b.stamps : nullptr;
    unsigned long long t0 = 0, t1 = 0;
    if (st) t0 = stamp();
    if (threadIdx.x == 0) bad[0] = 0.0;
    if (threadIdx.x < 4) pdone[threadIdx.x] = 0u;
    TileFetch<64, M, NTL> fa;
    TileFetch<16, M, NTL> frc;
    if (!TOP && sp == 0) {
        // first level: gather the block straight from the reduced band (no
        // pack launch), A, column tile w of C_i, row tile w of C_r and column
        // tile w of R_i, every load in flight first; and rows 16w.. of the
        // even blocks beside it (i - 1, and the last block when that is even)
        // to global memory for the later levels and the top
        constexpr int QA = M * M / NTL, QC = M * 16 / NTL;
        double va[QA], vc[QC], vr[QC], vz[QC];
        const BandCol col(b, P, radius, i, threadIdx.x % M);
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int e = threadIdx.x + q * NTL;
            va[q] = col.a(P, e / M, e % M);
        }
#pragma unroll
        for (int q = 0; q < QC; ++q) {
            const int e = threadIdx.x + q * NTL;
            vc[q] = pack_c(b, P, i, e / 16, 16 * w + e % 16);
            vr[q] = pack_c(b, P, r, 16 * w + e / M, e % M, hr);
            vz[q] = pack_r(b, P, i, e / 16, 16 * w + e % 16, hz);
        }
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int e = threadIdx.x + q * NTL;
            A[(e / M) * LD + e % M] = va[q];
        }
#pragma unroll
        for (int q = 0; q < QC; ++q) {
            const int e = threadIdx.x + q * NTL;
            Cc[(e / 16) * L16 + e % 16] = vc[q];
            Cr[(e / M) * LD + e % M] = vr[q];
            Rc[(e / 16) * L16 + e % 16] = vz[q];
        }
        pack_rows<NTL>(b, P, radius, i - 1, 16 * w, threadIdx.x);
        if (i + 1 == b.N - 1) pack_rows<NTL>(b, P, radius, i + 1, 16 * w, threadIdx.x);
    } else {   // every tile's loads in flight together, then the LDS stores
        // (C_i and C_r come from the neighbours' W blocks at every level after
        // the first: bgC / bgCr overwrite all of Cc and Cr, so they are not loaded)
        TileFetch<64, M, NTL> fwa, fwb;
        const bool hwb = i + sp < b.N;   // the neighbours' W blocks (the A update's operands)
        if (!TOP) fwa.fetch(b.Wr + (size_t)(i - sp) * M * M, M);
        if (hwb) fwb.fetch(b.Wl + (size_t)(i + sp) * M * M, M);
        fa.fetch(b.A + (size_t)i * M * M, M);
        if (hz) frc.fetch(b.R + (size_t)i * M * b.nrhs + 16 * w, b.nrhs);
        if (!TOP) fwa.put(Wa_l, M);
        if (hwb) fwb.put(Wb_l, M);
        fa.put(A, LD);
        if (hz) frc.put(Rc, L16);
    }
    __syncthreads();
    if (st) {
        t1 = stamp();
        if (threadIdx.x == 0) atomicAdd(st + 5, t1 - t0);   // loads
    }
    {
    // neighbours eliminated at stride sp: i-sp (always there) and i+sp.
    // A_i -= Wa' Wa + Wb' Wb (lower tiles), R_i[:, w] -= Wa' z_{i-sp}[:, w] +
    // Wb' z_{i+sp}[:, w], C_i[:, w] = -Wa' Wl_{i-sp}[:, w] and C_r's row tile
    // w = -(Wr_{i+sp}[:, w])' Wl_{i+sp}; then the factorisation.
    //
    // Just-in-time schedule (round 4).  fp64 MFMAs on a SIMD stall the
    // fp64 VALU of the pivot wave (wave 0) there, so wave 0's SIMD
    // partner (wave 4) issues no MFMA while a diagonal factor runs, and
    // the six helper waves (1-3, 5-7: SIMDs 1-3) do every tile product in
    // the four factor windows W0..W3, each tile's A update folded into
    // its trailing updates and done just before the panel or factor that
    // reads it, the R / C products spread over the windows' slack:
    //   S0  all waves: A_00's update as 8 one-chunk products
    //   W0  wave 0: A_00, diag16(0) | helpers: A updates of tiles (1,0),
    //       (2,0), (3,0), (1,1) as 8 half products (one per neighbour),
    //       C_0
    //   W1  wave 0: its own panel L_10 = (A_10 - halves) X_00', A_11
    //       (- halves - L_10 L_10'), diag16(1) | helpers: first the other
    //       panels L_20, L_30 (P(0), counted in LDS), then tiles (2,1),
    //       (3,1), (2,2) (A update + step 0), T_10, C_1..3
    //   W2 (P(1) first): tiles (3,2), (3,3) (A update + steps 0, 1), T_20,
    //       T_21, Cr
    //   W3 (P(2) first): T_30, T_31, T_32, R_0..2;  P3 with R_3 on wave 4
    // upd: the neighbours eliminated at stride sp update A / R / C (every
    // level but the first, whose blocks come straight from bcr_pack)
    const bool upd = sp > 0;
    // (TOP: no left neighbour -- its operands are never read, il is a placeholder)
    const int il = TOP ? i : i - sp, ir = i + sp;
    const bool hir = upd && ir < b.N;
    const double* Z1 = b.Z + (size_t)il * M * b.nrhs + 16 * w;
    const double* Z2 = b.Z + (size_t)ir * M * b.nrhs + 16 * w;
    const double* WL = b.Wl + (size_t)il * M * M + 16 * w;
    const double* WR = b.Wr + (size_t)ir * M * M + 16 * w;
    double* Wal = Wa_l;
    double* Wbl = Wb_l;
    // scratch tiles (LD layout): X's lower tiles until T_10 (window 1);
    // the tiles above the block diagonal of X and A, which nothing reads
    auto tile_at = [&](int sel, int r, int c) { return (sel ? X : A) + 16 * r * LD + 16 * c; };
    constexpr int8_t kS0[8][2] = {{1, 0}, {2, 0}, {3, 0}, {2, 1}, {3, 1}, {3, 2}, {0, 1}, {0, 2}};   // in X
    constexpr int8_t kHp[8][3] = {{0, 0, 1}, {0, 0, 2}, {0, 0, 3}, {0, 1, 2}, {0, 1, 3}, {0, 2, 3},
                                  {1, 0, 3}, {1, 1, 2}};   // (X?, r, c)
    auto hp = [&](int h) { return tile_at(kHp[h][0], kHp[h][1], kHp[h][2]); };
    constexpr int8_t kHt[4][2] = {{1, 0}, {2, 0}, {3, 0}, {1, 1}};   // half products: tile h / 2, neighbour h & 1
    auto half = [&](int h) {
        if (!upd) return;
        const int ti = kHt[h >> 1][0], tj = kHt[h >> 1][1];
        double* W = (h & 1) ? Wbl : Wal;
        if ((h & 1) && !hir) return;
        if (!(h & 1) && TOP) return;
        tile_st(hp(h), LD, 0, 0, mm_ll_rows<true, false, false>(zero4(), L3(W), M, 16 * ti, L3(W), M, 16 * tj, kM));
    };
    auto sub_halves = [&](v4d acc, int t) {   // acc - half a - half b of tile t (fixed order)
        if (!upd) return acc;
        if (!TOP) acc -= tile_ld(hp(2 * t), LD, 0, 0);
        if (hir) acc -= tile_ld(hp(2 * t + 1), LD, 0, 0);
        return acc;
    };
    // tile (ti, tj): its A update, then the trailing updates of steps 0..nk-1
    auto full = [&](int ti, int tj, int nk) {
        v4d acc = tile_ld(A, LD, 16 * ti, 16 * tj);
        if (upd && !TOP) acc = mm_ll_rows<true, false, true>(acc, L3(Wal), M, 16 * ti, L3(Wal), M, 16 * tj, kM);
        if (hir) acc = mm_ll_rows<true, false, true>(acc, L3(Wbl), M, 16 * ti, L3(Wbl), M, 16 * tj, kM);
        if (nk) acc = mm_ll<false, true, true>(acc, L3(A), LD, 16 * ti, L3(A), LD, 16 * tj, 0, 16 * nk);
        tile_st(A, LD, 16 * ti, 16 * tj, acc);
    };
    // T_nj = sum_{m=j..n-1} L_nm X_mj into X tile (n, j).  Of X = L^-1 this
    // workgroup needs only row tile w (stored for the back substitution) and
    // the rows above it that row w is formed from: the forward substitution
    // and the panels read X's diagonal tiles only.  Rows n > w are skipped
    // (C4: workgroup 0, which also carries the R column, forms none).
    auto tinv = [&](int n, int j) {
        if (n > w) return;
        tile_st(X, LD, 16 * n, 16 * j, mm_ll<false, false, false>(zero4(), L3(A), LD, 16 * n, L3(X), LD, 16 * j, 16 * j, 16 * n));
    };
    // neighbour products; g*: the global operands, fetched into registers by
    // the wave at the start of the window it runs them in (GTile)
    const bool hzu = hz && upd;
    auto bgR = [&](int v, const GTile& g1, const GTile& g2) {   // R_i[:, w] row tile v
        if (!hzu) return;
        v4d acc = tile_ld(Rc, L16, 16 * v, 0);
        if (!TOP) acc = mm_tr<true>(acc, L3(Wal), M, 16 * v, g1, kM);
        if (hir) acc = mm_tr<true>(acc, L3(Wbl), M, 16 * v, g2, kM);
        tile_st(Rc, L16, 16 * v, 0, acc);
    };
    auto bgC = [&](int v, const GTile& gl) {   // block (i, i-2sp) = (i, i-s)
        if (upd && !TOP) tile_st(Cc, L16, 16 * v, 0, mm_tr<true>(zero4(), L3(Wal), M, 16 * v, gl, kM));
    };
    auto bgCr = [&](int v, const GTile& gr) {   // block (r, r-s) = (r, i)
        if (hr && hir) tile_st(Cr, LD, 0, 16 * v, mm_rt<true>(zero4(), gr, L3(Wbl), M, 16 * v, kM));
    };
    auto fetch_z = [&](GTile& g1, GTile& g2) {
        if (!hzu) return;
        if (!TOP) g1.fetch(Z1, b.nrhs);
        if (hir) g2.fetch(Z2, b.nrhs);
    };
    auto fetch_wl = [&](GTile& g) {
        if (upd && !TOP) g.fetch(WL, M);
    };
    auto fetch_wr = [&](GTile& g) {
        if (hr && hir) g.fetch(WR, M);
    };
    // P(k), k >= 1: panels L_ik = A_ik X_kk' (i > k) and X_kj = -X_kk T_kj (j < k), waves 0..2
    auto pphase = [&](int k) {
        if (wave >= 3) return;
        if (wave >= 3 - k && k > w) return;   // X row tile k: not needed here (tinv)
        if (wave < 3 - k) {
            const int ii = k + 1 + wave;
            tile_st(A, LD, 16 * ii, 16 * k,
                    tile_mm<false, true, false>(zero4(), L3(A), LD, 16 * ii, L3(X), LD, 16 * k, 16 * k, 16 * k + 16));
        } else {
            const int j = wave - (3 - k);
            tile_st(X, LD, 16 * k, 16 * j,
                    tile_mm<false, false, true>(zero4(), L3(X), LD, 16 * k, L3(X), LD, 16 * j, 16 * k, 16 * k + 16));
        }
    };
    // diagnostic stamps (w == 0 workgroups, SFM_BCR_STAMPS): as chol_inv64
    unsigned long long* wmax = reinterpret_cast<unsigned long long*>(col);
    unsigned long long tf0 = 0, td = 0, tq = 0, tw = 0;
    if (st) {
        if (threadIdx.x < 8) wmax[threadIdx.x] = 0;
        tf0 = stamp();
    }
    auto wend = [&](int k) {
        if (st && (threadIdx.x & 63) == 0) atomicMax(wmax + (wave == 0 ? 4 : 0) + k, stamp() - tw);
    };
    // the pivot wave: A_nn's last update, then diag16(n)
    auto dfac = [&](int n, v4d acc) {
        unsigned long long ta = 0, tb = 0;
        if (st) ta = stamp();
        tile_st(A, LD, 16 * n, 16 * n, acc);
        wave_sync();
        if (st) tb = stamp();
        if (n == 3) diag16_last(np3, A + 16 * n * (LD + 1), X + 16 * n * (LD + 1), bad, col);
        else diag16(A + 16 * n * (LD + 1), X + 16 * n * (LD + 1), bad, col);
        if (st) {
            const unsigned long long te = stamp();
            td += te - ta;
            tq += te - tb;
        }
    };
    // ---- S0 -----------------------------------------------------------------
    {
        const int v = wave & 3;
        v4d part = zero4();
        if (wave < 4) {
            if (upd && !TOP) part = tile_mm<true, false, false>(part, L3(Wal), M, 0, L3(Wal), M, 0, 16 * v, 16 * v + 16);
        } else if (hir) part = tile_mm<true, false, false>(part, L3(Wbl), M, 0, L3(Wbl), M, 0, 16 * v, 16 * v + 16);
        if (upd) tile_st(tile_at(1, kS0[wave][0], kS0[wave][1]), LD, 0, 0, part);
    }
    __syncthreads();
    // ---- forward substitution of this workgroup's column tile w -------------
    // O_k = X_kk (B_k - sum_{m<k} L_km O_m), in place, for O = Wl[:, w]
    // (B = C_i[:, w] in Cc), Wr[:, w] (B = C_r[w, :]' in Cr, transposed) and
    // z[:, w] (B = R_i[:, w] in Rc): row tile k is formed as soon as the
    // factor's diagonal tile k is done, on the helper waves inside the next
    // window, instead of X C_i, X C_r', X R_i after the whole factorisation
    // (round 5: that tail was ~10k of a level's ~47k cycles).  fs(k): B_k -=
    // sum L_km O_m (L_km in A's lower tiles after P(m)); gs(k): O_k = X_kk B_k,
    // kept in LDS for the later row tiles and stored to global.
    double* const Wlg = b.Wl + (size_t)i * M * M;
    double* const Wrg = b.Wr + (size_t)i * M * M;
    double* const Zg = b.Z + (size_t)i * M * b.nrhs;
    auto fs_l = [&](double* B, int k) {   // B = Cc or Rc ([64][L16])
        v4d acc = tile_ld(B, L16, 16 * k, 0);
        acc = mm_ll<false, false, true>(acc, L3(A), LD, 16 * k, L3(B), L16, 0, 0, 16 * k);
        tile_st(B, L16, 16 * k, 0, acc);
    };
    auto gs_l = [&](double* B, int k, double* G, int ldg) {
        const v4d o = mm_ll<false, false, false>(zero4(), L3(X), LD, 16 * k, L3(B), L16, 0, 16 * k, 16 * k + 16);
        tile_st(B, L16, 16 * k, 0, o);
        tile_st(G, ldg, 16 * k, 16 * w, o);
        return o;
    };
    // TOP, fused: wave 7 accumulates block 0's corner partial z_0' z_0 (column
    // tile 0) from each row tile of z_0 as it forms it -- register r of the
    // MFMA result holds rows 16k + kk + 4r, i.e. k-step 4k + r of the corner
    // body's own product, in the same order (bit-identical)
    v4d qz = zero4();
    const bool q_here = TOP && w == 0 && gridDim.x > 4;
    auto fs_r = [&](int k) {   // Cr(0, k) -= sum_m Cr(0, m) L_km'
        v4d acc = tile_ld(Cr, LD, 0, 16 * k);
        acc = mm_ll<false, true, true>(acc, L3(Cr), LD, 0, L3(A), LD, 16 * k, 0, 16 * k);
        tile_st(Cr, LD, 0, 16 * k, acc);
    };
    auto gs_r = [&](int k) {   // Cr(0, k) = Cr(0, k) X_kk' = O_k'; Wr rows 16k.. (transposed store)
        const v4d o = tile_mm<false, true, false>(zero4(), L3(Cr), LD, 0, L3(X), LD, 16 * k, 16 * k, 16 * k + 16);
        tile_st(Cr, LD, 0, 16 * k, o);
        const int lane = threadIdx.x & 63, li = lane & 15, kk = lane >> 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) Wrg[(16 * k + li) * M + 16 * w + kk + 4 * q] = o[q];
    };
    // gs of row tile k on waves 5-7 in the P(k) phase, right after the
    // window that produced X_kk (those waves are idle there); fs of row tile
    // k + 1 in window k + 1, after P(k) gave L_{k+1,k}
    auto gs_k = [&](int k) {
        if (wave == 5) {
            if (!TOP) gs_l(Cc, k, Wlg, M);
        } else if (wave == 6 && hr) {
            gs_r(k);
        } else if (wave == 7 && hz) {
            const v4d o = gs_l(Rc, k, Zg, b.nrhs);
            if (q_here) {
#pragma unroll
                for (int r = 0; r < 4; ++r) qz = __builtin_amdgcn_mfma_f64_16x16x4f64(o[r], o[r], qz, 0, 0, 0);
            }
        }
    };
    auto fs_lk = [&](int k) {
        if (!TOP) fs_l(Cc, k);
    };
    auto fs_zk = [&](int k) {
        if (hz) fs_l(Rc, k);
    };
    auto fs_rk = [&](int k) {
        if (hr) fs_r(k);
    };
    // this workgroup's row tile w of X for the back substitution (final after P(w))
    auto store_x = [&](int nth, int t0) {
        double* Xg = b.L + (size_t)i * M * M + 16 * w * M;
        for (int e = t0; e < 16 * M; e += nth) Xg[e] = X[(16 * w + e / M) * LD + e % M];
    };
    // ---- W0 -----------------------------------------------------------------
    // (helpers: the A update halves, and every neighbour product of C_i, C_r
    // and R_i that the forward substitution needs by window 1 or 2)
    if (st) tw = stamp();
    switch (wave) {
        case 0: {
            v4d acc = tile_ld(A, LD, 0, 0);
            if (upd) {
#pragma unroll
                for (int q = 0; q < NWL; ++q) acc -= tile_ld(tile_at(1, kS0[q][0], kS0[q][1]), LD, 0, 0);
            }
            dfac(0, acc);
            break;
        }
        case 1: { GTile z1, z2; fetch_z(z1, z2); half(0); half(3); bgR(0, z1, z2); break; }
        case 2: { GTile z1, z2; fetch_z(z1, z2); half(1); half(4); bgR(1, z1, z2); break; }
        case 3: { GTile z1, z2; fetch_z(z1, z2); half(2); bgR(2, z1, z2); break; }
        case 5: { GTile g; fetch_wr(g); half(6); bgCr(0, g); break; }
        case 6: { GTile g; fetch_wr(g); half(7); bgCr(1, g); break; }
        case 7: { GTile g; fetch_wl(g); half(5); bgC(0, g); bgC(1, g); break; }
        default: break;
    }
    wend(0);
    __syncthreads();
    // ---- window hand-offs without a P phase (round 5) ------------------------
    // P(k)'s products (the panels L_ik = A_ik X_kk', the inverse's row tile k,
    // the forward substitution's G steps) run at the start of window k + 1
    // instead of in a phase of their own between two barriers: the pivot
    // wave forms its own panel L_{k+1,k} = (X_kk A_{k+1,k}')' as an MFMA
    // result whose registers are at once the operands of A_{k+1,k+1} -=
    // L L' (no LDS round trip, no barrier before its next diagonal factor).
    // Each wave publishes its P(k) item as bit `wave` of pdone[k], and each
    // window product waits for the bits of exactly the items it reads
    // (products with no P(k) input run before the wait).
    auto p_sig = [&](int k) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or(pdone + k, 1u << wave, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto p_wait = [&](int k, unsigned bits) {
        while ((__hip_atomic_load(pdone + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & bits) != bits)
            __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    };
    constexpr unsigned kL = 1u, kW1 = 2u, kW2 = 4u, kW7 = 128u;   // L_{k+1,k} (wave 0), waves 1, 2, 7's items
    // P(k)'s item of wave 1 or 2: a panel L_ik (k = 0: its A update's halves
    // first) or an inverse tile X_kj = -X_kk T_kj; then its bit
    auto p_item = [&](int k) {
        if (wave < 3 - k) {
            const int ii = k + 1 + wave;
            if (k == 0) {
                tile_st(A, LD, 16 * ii, 0, sub_halves(tile_ld(A, LD, 16 * ii, 0), wave));
                wave_sync();
            }
            tile_st(A, LD, 16 * ii, 16 * k,
                    tile_mm<false, true, false>(zero4(), L3(A), LD, 16 * ii, L3(X), LD, 16 * k, 16 * k, 16 * k + 16));
        } else if (k <= w) {   // X row tile k: not needed here otherwise (tinv)
            const int j = wave - (3 - k);
            tile_st(X, LD, 16 * k, 16 * j,
                    tile_mm<false, false, true>(zero4(), L3(X), LD, 16 * k, L3(X), LD, 16 * j, 16 * k, 16 * k + 16));
        }
        p_sig(k);
    };
    // waves 5-7: P(k)'s G steps, then their bits
    auto p_g = [&](int k) {
        gs_k(k);
        p_sig(k);
    };
    // the pivot wave between diagonal factors k and k + 1
    auto self_panel = [&](int k, v4d c) {
        const int n = k + 1;
        if (k == 0) {   // L_10's A update (the halves of tile (1, 0))
            tile_st(A, LD, 16, 0, sub_halves(tile_ld(A, LD, 16, 0), 0));
            wave_sync();
        }
        // Y = L_{n,k}' = X_kk A_{n,k}': element (kk + 4r, i) in register r
        const v4d y = tile_mm<false, true, false>(zero4(), L3(X), LD, 16 * k, L3(A), LD, 16 * n, 16 * k, 16 * k + 16);
        {   // L_{n,k} (= Y') for the helpers: transposed store, then the bit
            const int lane = threadIdx.x & 63, li = lane & 15, kk = lane >> 4;
#pragma unroll
            for (int r = 0; r < 4; ++r) A[(16 * n + li) * LD + 16 * k + kk + 4 * r] = y[r];
        }
        p_sig(k);
        // A_nn -= L L' = Y' Y: the MFMA A operand of Y' and the B operand of Y
        // are Y's own accumulator registers
#pragma unroll
        for (int r = 0; r < 4; ++r) c = __builtin_amdgcn_mfma_f64_16x16x4f64(-y[r], y[r], c, 0, 0, 0);
        dfac(n, c);
    };
    // ---- W1 -----------------------------------------------------------------
    if (st) tw = stamp();
    switch (wave) {
        case 0: self_panel(0, sub_halves(tile_ld(A, LD, 16, 16), 3)); break;
        case 1: p_item(0); p_wait(0, kL); full(2, 1, 1); break;                    // L_20
        case 2: p_item(0); p_wait(0, kL); full(3, 1, 1); break;                    // L_30
        case 3: p_wait(0, kW1); full(2, 2, 1); break;
        case 5: { p_g(0); GTile g; fetch_wl(g); bgC(2, g); p_wait(0, kL); fs_lk(1); break; }
        case 6: p_g(0); p_wait(0, kL); fs_rk(1); p_wait(0, kW7); fs_zk(1); break;
        case 7: { p_g(0); GTile g; fetch_wr(g); bgCr(2, g); p_wait(0, kL); tinv(1, 0); break; }
        default: break;
    }
    wend(1);
    __syncthreads();
    // ---- W2 -----------------------------------------------------------------
    if (st) tw = stamp();
    switch (wave) {
        case 0: self_panel(1, tile_ld(A, LD, 32, 32)); break;
        case 1: p_item(1); p_wait(1, kL); full(3, 2, 2); break;                    // L_31
        case 2: p_item(1); p_wait(1, kW1); full(3, 3, 2); break;                   // X_10
        case 3: p_wait(1, kL | kW2); tinv(2, 0); tinv(2, 1); break;
        case 5: p_g(1); p_wait(1, kL); fs_lk(2); break;
        case 6: p_g(1); p_wait(1, kL); fs_rk(2); break;
        case 7: { p_g(1); GTile z1, z2; fetch_z(z1, z2); bgR(3, z1, z2); p_wait(1, kL); fs_zk(2); break; }
        default: break;
    }
    wend(2);
    __syncthreads();
    // ---- W3 -----------------------------------------------------------------
    if (st) tw = stamp();
    switch (wave) {
        case 0: self_panel(2, tile_ld(A, LD, 48, 48)); break;
        case 1: p_item(2); p_wait(2, kL); tinv(3, 0); break;                       // X_20
        case 2: p_item(2); p_wait(2, kL); tinv(3, 1); break;                       // X_21
        case 3: p_wait(2, kL); tinv(3, 2); break;
        case 4:   // no MFMA on the pivot wave's SIMD; row tile 2 of X is final with X_20, X_21
            if (w < 3) {
                if (w == 2) p_wait(2, kW1 | kW2);
                store_x(64, threadIdx.x & 63);
            }
            break;
        case 5: { p_g(2); GTile g; fetch_wl(g); bgC(3, g); p_wait(2, kL); fs_lk(3); break; }
        case 6: { p_g(2); GTile g; fetch_wr(g); bgCr(3, g); p_wait(2, kL); fs_rk(3); break; }
        case 7: p_g(2); p_wait(2, kL); fs_zk(3); break;
        default: break;
    }
    wend(3);
    __syncthreads();
    // ---- P3: X's last row tile; the last row tile of every output -----------
    pphase(3);
    gs_k(3);
    if (q_here && wave == 7) corner_put_lds(P, qz, Cc);   // block 0's corner partial (Cc: unused by the top)
    if (st && threadIdx.x == 0) {
        atomicAdd(st + 0, td);
        atomicAdd(st + 1, stamp() - tf0);
        atomicAdd(st + 7, tq);
        for (int q = 0; q < 8; ++q) atomicAdd(st + 8 + q, wmax[q]);
    }
    if (w == 3) {
        __syncthreads();   // X_3j of P3
        store_x(NTL, threadIdx.x);
    }
    }
    if (threadIdx.x == 0 && bad[0] != 0.0) b.fail[0] = 1.0;
    if constexpr (TOP) {
        // fused launch: block 0's corner partial is in LDS (wave 7, above);
        // the rest's tagged sum, then the corner solve (bcr_corner_body)
        if (w == 0 && gridDim.x > 4) {
            __syncthreads();
            bcr_corner_body(b, P, radius, 0, true, true, epoch, Cc);
        }
        return;
    }
    if (st) {
        __syncthreads();
        if (threadIdx.x == 0) atomicAdd(st + 6, stamp() - t0);   // through the X copy
    }
    if (st) {
        __syncthreads();
        if (threadIdx.x == 0) {
            atomicAdd(st + 2, t1 - t0);              // loads + update
            atomicAdd(st + 3, stamp() - t0);         // whole block
            atomicAdd(st + 4, 1ull);
        }
    }
}

// ---- top: super-block 0 alone; y_0 = X' X R_0 ----------------------------------
// sp > 0: first block 0's update from its right neighbour sp, eliminated by
// the last level (A_0 -= Wl_sp' Wl_sp, R_0 -= Wl_sp' z_sp; lower tiles only).
__device__ __forceinline__ void bcr_top_body(const BcrArgs& b, int sp, double* sm) {
    const int ldr = b.nrhs + 1, kM = bcr_kM(b);
    double* A = sm;
    double* X = A + M * LD;
    double* R = X + M * LD;
    double* T = R + M * ldr;
    double* Wb = T + M * ldr;       // [64][LD] Wl_sp
    double* Zb = Wb + M * LD;       // [64][ldr] z_sp
    double* sc = Zb + M * ldr;
    double* bad = sc + 33;
    const int wave = threadIdx.x >> 6;
    const bool upd = sp > 0 && sp < b.N;
    if (threadIdx.x == 0) bad[0] = 0.0;
    auto loads = [&](auto ncz) {   // every tile's loads in flight together
        constexpr int NCZ = decltype(ncz)::value;
        TileFetch<64, M, NTL> fa, fwb;
        TileFetch<NCZ, M, NTL> fr, fzb;
        fa.fetch(b.A, M);
        fr.fetch(b.R, b.nrhs);
        if (upd) {
            fwb.fetch(b.Wl + (size_t)sp * M * M, M);
            fzb.fetch(b.Z + (size_t)sp * M * b.nrhs, b.nrhs);
        }
        fa.put(A, LD);
        fr.put(R, ldr);
        if (upd) {
            fwb.put(Wb, LD);
            fzb.put(Zb, ldr);
        }
    };
    if (b.nrhs == 16) loads(std::integral_constant<int, 16>{});
    else loads(std::integral_constant<int, 32>{});
    for (int e = threadIdx.x; e < M * LD; e += NTL) X[e] = 0.0;
    __syncthreads();
    if (upd) {
        // A_0 -= Wb' Wb (lower tiles) and R_0 -= Wb' z_sp: wave 0 updates A_00 and
        // goes on to its diagonal factor, waves 1..7 do the other 9 tiles and
        // the R row tiles meanwhile (as bcr_level_kernel)
        auto a_tile = [&](int q) {
            const int ti = q < 1 ? 0 : q < 3 ? 1 : q < 6 ? 2 : 3;
            const int tj = q - ti * (ti + 1) / 2;
            v4d acc = tile_ld(A, LD, 16 * ti, 16 * tj);
            acc = mm_ll_rows<true, false, true>(acc, L3(Wb), LD, 16 * ti, L3(Wb), LD, 16 * tj, kM);
            tile_st(A, LD, 16 * ti, 16 * tj, acc);
        };
        const int nrt = b.nrhs / 16;
        {   // A_00's update: its 4 k-chunk products on waves 0..3 (X rows 16..63 free until P(1))
            double* scr = X + 16 * LD;
            if (wave < 4)
                tile_st(scr + 256 * wave, 16, 0, 0,
                        tile_mm<true, false, false>(zero4(), Wb, LD, 0, Wb, LD, 0, 16 * wave, 16 * wave + 16));
        }
        __syncthreads();
        auto pre0 = [&] {
            const double* scr = X + 16 * LD;
            v4d acc = tile_ld(A, LD, 0, 0);
#pragma unroll
            for (int q = 0; q < 4; ++q) acc -= tile_ld(scr + 256 * q, 16, 0, 0);
            tile_st(A, LD, 0, 0, acc);
        };
        auto preN = [&] {
            for (int t = wave - 1; t < 9 + 4 * nrt; t += NWL - 1) {
                if (t < 9) {
                    a_tile(t + 1);
                } else {
                    const int v = (t - 9) / nrt, tj = (t - 9) % nrt;
                    v4d acc = tile_ld(R, ldr, 16 * v, 16 * tj);
                    acc = mm_ll_rows<true, false, true>(acc, L3(Wb), LD, 16 * v, L3(Zb), ldr, 16 * tj, kM);
                    tile_st(R, ldr, 16 * v, 16 * tj, acc);
                }
            }
        };
        chol_inv64<NWL>(A, X, bad, sc, nullptr, pre0, preN, NoBg(), 6 * b.K - 48);
    } else {
        chol_inv64<NWL>(A, X, bad, sc, nullptr, NoPre(), NoPre(), NoBg(), 6 * b.K - 48);
    }
    if (threadIdx.x == 0 && bad[0] != 0.0) b.fail[0] = 1.0;
    // the root's forward solve z_0 = X R_0, every column (the corner system
    // reduces the arrow's, bcr_corner_kernel), and X_0 for the back substitution
    if (wave < 4) {
        for (int tj = 0; tj < b.nrhs / 16; ++tj)
            tile_st(b.Z, b.nrhs, 16 * wave, 16 * tj,
                    mm_ll<false, false, false>(zero4(), L3(X), LD, 16 * wave, L3(R), ldr, 16 * tj, 0, 16 * (wave + 1)));
    } else {
        for (int e = threadIdx.x - 256; e < M * M; e += NTL - 256) b.L[e] = X[(e / M) * LD + e % M];
    }
}

__global__ __launch_bounds__(NTL) void bcr_top_kernel(BcrArgs b, int sp) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    bcr_top_body(b, sp, sm);
}

// ---- bordered arrow, corner first ---------------------------------------------
// The forward levels (and the top) leave every block's z_i = X_i R_i, all
// columns: the rhs and the arrow's.  With B = L L' the band's CR
// factorisation (blocks in elimination order), E' B^-1 E = sum_i z_i[:, E]'
// z_i[:, E] and E' B^-1 r = sum_i z_i[:, E]' z_i[:, 0], so the corner system
//   (S_c + D^2 - E' B^-1 E) x_c = rhs_c - E' B^-1 r
// is formed before any back substitution, which then carries one column,
//   z'_i = z_i[:, 0] - z_i[:, E] x_c   (the forward solve of r - E x_c),
// instead of the 1 + na columns (padded to 16) a bordered back substitution
// carries.  One workgroup per block: wave 0 forms Q_i = z_i' z_i on the MFMA
// and stores its rows 1..na, columns 0..na; the last workgroup to finish (an
// agent-scope counter, which it resets) adds the partials in block order
// and solves the corner.
// (z_fresh: this workgroup wrote z_I itself just before -- the top, in the
// fused launch -- so wave 0 reads it write-through, past this CU's L1)
__device__ __forceinline__ void bcr_corner_body(const BcrArgs& b, const DevProblem& P, double radius, int I,
                                                bool z_fresh, bool part_done, unsigned tag, const double* own) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int na = P.iw * P.nintr, iw = P.iw;   // bordered columns (<= 16)
    constexpr int kQ = 17;                      // part row stride: columns 0..16
    __shared__ double Mc[16 * 16 + 16];
    __shared__ int last;
    unsigned* counter = reinterpret_cast<unsigned*>(b.fail + 4);
    if (wave == 0 && !part_done) {
        const int i = lane & 15, kk = lane >> 4, ntc = b.nrhs / 16;
        const double* Z = b.Z + (size_t)I * M * b.nrhs;
        double z0[16], z1[16];   // z[4 ks + kk][i], z[4 ks + kk][16 + i]: every load issued first
        if (z_fresh) {
#pragma unroll
            for (int ks = 0; ks < 16; ++ks) z0[ks] = ld_sc1(Z + (4 * ks + kk) * b.nrhs + i);
            if (ntc > 1) {
#pragma unroll
                for (int ks = 0; ks < 16; ++ks) z1[ks] = ld_sc1(Z + (4 * ks + kk) * b.nrhs + 16 + i);
            }
        } else {
#pragma unroll
            for (int ks = 0; ks < 16; ++ks) z0[ks] = Z[(4 * ks + kk) * b.nrhs + i];
            if (ntc > 1) {
#pragma unroll
                for (int ks = 0; ks < 16; ++ks) z1[ks] = Z[(4 * ks + kk) * b.nrhs + 16 + i];
            }
        }
        v4d q00 = zero4(), q10 = zero4(), q11 = zero4();
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) q00 = __builtin_amdgcn_mfma_f64_16x16x4f64(z0[ks], z0[ks], q00, 0, 0, 0);
        if (ntc > 1) {
#pragma unroll
            for (int ks = 0; ks < 16; ++ks) {
                q10 = __builtin_amdgcn_mfma_f64_16x16x4f64(z1[ks], z0[ks], q10, 0, 0, 0);
                q11 = __builtin_amdgcn_mfma_f64_16x16x4f64(z1[ks], z1[ks], q11, 0, 0, 0);
            }
        }
        // element (row kk + 4r, column i) of each tile; keep rows 1..na, columns 0..na
        corner_put(b, P, I, q00, q10, q11, ntc);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // the partials are stored write-through (sc1) and drained above: a
    // relaxed ticket publishes them, and a last arriver reads them with sc1
    // loads (no release or acquire fence: Guideline 16, counter form).
    // Two tickets (round 5): the last of blocks 1..N-1 sums their partials
    // into slot N -- in the fused launch while workgroup 0 still factors the
    // top -- and takes the second ticket, as does block 0 with its own
    // partial; the last of those two adds slot 0 + slot N and solves.  (One
    // ticket over all N left the N-partial sum to workgroup 0, after the top.)
    unsigned* counter2 = reinterpret_cast<unsigned*>(b.fail + 6);
    const int el = threadIdx.x >> 3, g = threadIdx.x & 7;   // 32 elements x 8 lanes per pass
    const int nel = na * kQ;                                // partial doubles: rows 1..na, columns 0..na
    __syncthreads();
    bool rest_sum = false;
    if (I > 0) {
        if (threadIdx.x == 0)
            last = __hip_atomic_fetch_add((gu32*)counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   (unsigned)b.N - 2;
        __syncthreads();
        if (!last) return;
        if (threadIdx.x == 0) __hip_atomic_store((gu32*)counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        rest_sum = true;
    }
    if (rest_sum) {
        // blocks [1 + g (N-1)/8, 1 + (g+1) (N-1)/8) per lane, the 8 lanes of an
        // element then combined by a fixed xor butterfly (deterministic)
        const int nr = b.N - 1;
        for (int base = 0; base < nel && (int)threadIdx.x < NT; base += NT / 8) {
            const int k = base + el;
            const int J0 = 1 + nr * g / 8, J1 = 1 + nr * (g + 1) / 8;
            double t = 0.0;
            if (k < nel) {
#pragma unroll 4
                for (int J = J0; J < J1; ++J) t += ld_sc1(b.part + (size_t)J * 512 + k);
            }
#pragma unroll
            for (int o = 1; o < 8; o <<= 1) t += __shfl_xor(t, o);
            if (g == 0 && k < nel) {
                if (tag) put_y(reinterpret_cast<unsigned long long*>(b.part + (size_t)b.N * 512), k, t, tag);
                else st_sc1(b.part + (size_t)b.N * 512 + k, t);
            }
        }
        if (tag) return;   // (the fused top's workgroup 0 polls the tagged sums and solves)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (!tag) {
        if (threadIdx.x == 0)
            last = __hip_atomic_fetch_add((gu32*)counter2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   (b.N > 1 ? 1u : 0u);
        __syncthreads();
        if (!last) return;
        if (threadIdx.x == 0) __hip_atomic_store((gu32*)counter2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // Tagged (the fused top, round 5): workgroup 0 always solves.  Its own
    // partial never left the workgroup (own: LDS, as wave 7 formed it), and the
    // rest's sum arrives as {tag, 32 bits} granules (the data is the flag, as
    // the back substitution's y) -- no drain, no ticket, one poll.
    const unsigned long long* rest_g = reinterpret_cast<const unsigned long long*>(b.part + (size_t)b.N * 512);
    auto rest_tagged = [&](int off) {
        unsigned lo = 0, hi = 0;
        for (unsigned spins = 0;; ++spins) {
            const unsigned long long x0 = __hip_atomic_load((gu64*)(rest_g + 2 * off), __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long x1 = __hip_atomic_load((gu64*)(rest_g + 2 * off + 1), __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
            lo = (unsigned)x0;
            hi = (unsigned)x1;
            if ((unsigned)(x0 >> 32) == tag && (unsigned)(x1 >> 32) == tag) break;
            __builtin_amdgcn_s_sleep(1);
            if (spins > (1u << 22)) {   // ~ seconds: a lost producer, never a normal wait
                st_sc1(b.fail + 1, 1.0);
                break;
            }
        }
        return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
    };
    auto sum_parts = [&](int off) {   // block 0's partial + the rest's sum (slot N)
        if (tag) return own[off] + rest_tagged(off);
        const double t0 = ld_sc1(b.part + off);
        return b.N > 1 ? t0 + ld_sc1(b.part + (size_t)b.N * 512 + off) : t0;
    };
    for (int k = threadIdx.x; k < na * na + na; k += blockDim.x) {
        if (k < na * na) {
            const int a = k / na, c = k % na;   // lower triangle (a >= c), mirrored
            if (a >= c) {
                const double red = sum_parts(a * kQ + c + 1);
                double m = P.Scorner[(((size_t)(a / iw) * P.nintr + c / iw) * iw * iw) + (a % iw) * iw + c % iw];
                if (a == c) {
                    const double lm = sqrt(clampd(P.cnF[P.nb + a], P.min_diag, P.max_diag) / radius);
                    m += lm * lm;
                }
                Mc[a * 16 + c] = m - red;
            }
        } else {
            const int a = k - na * na;
            Mc[256 + a] = P.rhs[P.nb + a] - sum_parts(a * kQ);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        // dense Cholesky solve of the corner (<= 16 x 16, lower triangle)
        bool ok = true;
        for (int j = 0; j < na; ++j) {
            double d = Mc[j * 16 + j];
            for (int k = 0; k < j; ++k) d -= Mc[j * 16 + k] * Mc[j * 16 + k];
            if (!(d > 0.0)) ok = false;
            d = sqrt(d);
            Mc[j * 16 + j] = d;
            for (int i2 = j + 1; i2 < na; ++i2) {
                double t = Mc[i2 * 16 + j];
                for (int k = 0; k < j; ++k) t -= Mc[i2 * 16 + k] * Mc[j * 16 + k];
                Mc[i2 * 16 + j] = t / d;
            }
        }
        double* v = Mc + 256;
        for (int i2 = 0; i2 < na; ++i2) {
            double t = v[i2];
            for (int k = 0; k < i2; ++k) t -= Mc[i2 * 16 + k] * v[k];
            v[i2] = t / Mc[i2 * 16 + i2];
        }
        for (int i2 = na - 1; i2 >= 0; --i2) {
            double t = v[i2];
            for (int k = i2 + 1; k < na; ++k) t -= Mc[k * 16 + i2] * v[k];
            v[i2] = t / Mc[i2 * 16 + i2];
            P.yF[P.nb + i2] = v[i2];
        }
        if (!ok) b.fail[0] = 1.0;
    }
}

__global__ __launch_bounds__(NT) void bcr_corner_kernel(BcrArgs b, DevProblem P, double radius) {
    bcr_corner_body(b, P, radius, blockIdx.x, false);
}

// top + corner in one launch: workgroup 0 solves the top system (z_0, X_0)
// and then adds its corner partial; the other workgroups add theirs at once
// (their z_i are final since the levels).
// Untagged (bcr_corner_kernel after a separate top launch): the last to
// arrive solves the corner and no workgroup waits for another.
// Tagged (the default fused top): workgroup 0 always solves, and it WAITS for
// the rest's tagged corner sums (slot N), which the last of workgroups
// 1..N-1 to take the ticket writes (bcr_corner_body).  This is the one wait
// in the file that runs against the lower-index rule: it relies on
// workgroups 1..N-1 making progress while workgroup 0 spins.  They never wait on anything (their inputs are
// final before the launch), so they finish as soon as they are resident; a
// held CU only delays them.  The spin is bounded (2^22 polls with s_sleep 1,
// about seconds) and reports a lost producer as SFM_ERR_DEVICE (fail[1])
// instead of hanging.  tests/test_ba_general_gpu.py::test_band_solve_under_contention
// runs this path (and the split path) while another context holds the CUs.
__global__ __launch_bounds__(NTL) void bcr_top_corner_kernel(BcrArgs b, DevProblem P, double radius, int sp) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    if (blockIdx.x == 0) {
        bcr_top_body(b, sp, sm);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // z_0 written (read back write-through)
        __syncthreads();
    }
    bcr_corner_body(b, P, radius, blockIdx.x, blockIdx.x == 0);
}

// ---- back substitution, one column --------------------------------------------
//   y_i = X_i' (z'_i - Wl_i y_{i-s} - Wr_i y_{i+s}),  z'_i = z_i[:, 0] - z_i[:, E] x_c
// for block i eliminated at stride s (the root, block 0: no neighbours); its
// real rows go to yF.  256 threads: thread (row, p) takes 32 of the row's 128
// [Wl | Wr] coefficients, then 16 of the rows of X' (X staged in LDS);
// four-lane sums in a fixed order.
// FLOW: every block of every level in one launch, top-down (workgroup k waits
// only for workgroups < k, so any residency makes progress).  y_i (64
// doubles) is handed over as 128 tagged granules {epoch, 32 bits} stored
// write-through (Guideline 16 R2: the data is the flag, no fence either
// side): a consumer's wave 0 re-reads its neighbours' granules until every
// tag holds this solve's epoch, after staging everything the forward pass
// left.  The last workgroup to finish publishes the solve verdict.
constexpr int kYG = 128;   // granules per block
__device__ __forceinline__ void put_y(unsigned long long* g, int row, double v, unsigned epoch) {
    const unsigned long long bits = (unsigned long long)__double_as_longlong(v), tag = (unsigned long long)epoch << 32;
    __hip_atomic_store((gu64*)(g + 2 * row), tag | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gu64*)(g + 2 * row + 1), tag | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// wave 0: granules of y_a (and y_b) into LDS dst_a / dst_b as doubles
__device__ __forceinline__ void get_y(const unsigned long long* ga, const unsigned long long* gb, double* dst_a,
                                      double* dst_b, unsigned epoch, double* fail) {
    const int lane = threadIdx.x & 63;
    unsigned va[2], vb[2];
    for (unsigned spins = 0;;) {
        bool ok = true;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const unsigned long long x = __hip_atomic_load((gu64*)(ga + lane + 64 * h), __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
            va[h] = (unsigned)x;
            ok &= (unsigned)(x >> 32) == epoch;
            if (gb) {
                const unsigned long long y = __hip_atomic_load((gu64*)(gb + lane + 64 * h), __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT);
                vb[h] = (unsigned)y;
                ok &= (unsigned)(y >> 32) == epoch;
            }
        }
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) {   // ~ seconds: a lost producer, never a normal wait
            if (lane == 0) st_sc1(fail + 1, 1.0);   // a wait timeout, not a numerical failure
            break;
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        reinterpret_cast<unsigned*>(dst_a)[lane + 64 * h] = va[h];   // little endian: granule 2j = low word of y_j
        if (gb) reinterpret_cast<unsigned*>(dst_b)[lane + 64 * h] = vb[h];
    }
}

// The LM candidate of the block's cameras (BcrCand; round 5): as soon as y_i
// is known, threads 0..K-1 each form one camera's candidate extrinsics and
// CamPre with cand_kernel's arithmetic (ba_cand.h; their current values and
// column scales loaded at the start, during the wait), and the block's norm
// partial goes to part_f[i] (cameras in block order); the root also forms the
// intrinsics' candidates (part_f[N]) and copies the images without camera
// columns.  cand_kernel's launch and its dependent global round trips leave
// the iteration (its ~8 us at C4 and at rank 0 of N = 8).
template <bool FLOW>
__global__ __launch_bounds__(NT) void bcr_back_kernel(BcrArgs b, DevProblem P, int s_arg, unsigned epoch,
                                                      BcrCand cand) {
    __shared__ double Xs[M * LD];
    __shared__ double u[M];
    __shared__ double yl[M], yr[M];
    __shared__ double yc[M];
    __shared__ double redc[16][3];
    int i = -1, s = 0;
    if (FLOW) {   // workgroup k: the root, then the odd blocks of s_top / 2, ..., 1
        int k = blockIdx.x;
        if (k == 0) {
            i = 0;
        } else {
            --k;
            for (s = s_arg / 2; s >= 1; s >>= 1) {
                const int n_odd = (b.N - s + 2 * s - 1) / (2 * s);
                if (k < n_odd) {
                    i = s + 2 * s * k;
                    break;
                }
                k -= n_odd;
            }
        }
    } else {      // one level: s_arg = 0 the root, else its odd blocks
        s = s_arg;
        i = s == 0 ? (blockIdx.x == 0 ? 0 : -1) : s + 2 * s * (int)blockIdx.x;
    }
    unsigned long long* Yg = reinterpret_cast<unsigned long long*>(b.Y);   // [N][kYG] granules
    const int t = threadIdx.x, row = t >> 2, p = t & 3;
    const bool valid = i >= 0 && i < b.N;
    if (valid) {
        const int l = i - s, r = i + s;
        const bool hl = s > 0, hr = s > 0 && r < b.N;
        const bool use = p < 2 ? hl : hr;
        // this thread's camera (t < K) for the candidate: current values and
        // column terms first, so their round trips overlap the wait for y
        const int cb = i * b.K + t;
        const bool cam = t < b.K && cb < P.ncam;
        int cimg = 0;
        double cx[6], csf[6], cbf[6];
        if (cam) {
            cimg = P.blk_img[cb];
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                csf[a] = P.scaleF[6 * (size_t)cb + a];
                cbf[a] = P.bF[6 * (size_t)cb + a];
                cx[a] = cand.extr[6 * (size_t)cimg + a];
            }
        }
        // everything of the forward pass first: this row's [Wl | Wr]
        // coefficients, X into LDS, and z'_row
        double w[32];
        if (use) {
            const double2* src = reinterpret_cast<const double2*>(
                (p < 2 ? b.Wl : b.Wr) + (size_t)i * M * M + row * M + 32 * (p & 1));
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const double2 v = src[q];
                w[2 * q] = v.x;
                w[2 * q + 1] = v.y;
            }
        }
        load_tile<64, M, NT>(Xs, LD, b.L + (size_t)i * M * M, M);
        double zr = 0.0;
        if (p == 0) {
            const double* z = b.Z + ((size_t)i * M + row) * b.nrhs;
            const double* xc = P.yF + P.nb;
            zr = z[0];
            for (int a = 0; a < P.iw * P.nintr; ++a) zr -= z[1 + a] * xc[a];
        }
        if (hl) {
            if (t < 64) {
                if (FLOW) get_y(Yg + (size_t)l * kYG, hr ? Yg + (size_t)r * kYG : nullptr, yl, yr, epoch, b.fail);
                else {   // an earlier launch wrote them
                    for (int e = t; e < 2 * kYG; e += 64) {
                        const bool right = e >= kYG;
                        if (right && !hr) break;
                        reinterpret_cast<unsigned*>(right ? yr : yl)[e & (kYG - 1)] =
                            (unsigned)Yg[(size_t)(right ? r : l) * kYG + (e & (kYG - 1))];
                    }
                }
            }
        }
        __syncthreads();
        double acc = 0.0;
        if (use) {   // four independent chains (a 32-long dependent fma chain was on the path)
            const double* y = (p < 2 ? yl : yr) + 32 * (p & 1);
            double c4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int q = 0; q < 32; ++q) c4[q & 3] = fma(w[q], y[q], c4[q & 3]);
            acc = (c4[0] + c4[1]) + (c4[2] + c4[3]);
        }
        acc += __shfl_xor(acc, 1);   // (p0 + p1) + (p2 + p3): the same on the four lanes
        acc += __shfl_xor(acc, 2);
        if (p == 0) u[row] = zr - acc;
        __syncthreads();
        // y_j = sum_r X_rj u_r over X's lower tiles (its diagonal tiles carry
        // exact zeros above the diagonal; the tiles above are never written)
        double a2 = 0.0;
        if (p >= (row >> 4)) {   // (two independent chains)
            double c2[2] = {0.0, 0.0};
#pragma unroll
            for (int q = 0; q < 16; ++q) c2[q & 1] = fma(Xs[(16 * p + q) * LD + row], u[16 * p + q], c2[q & 1]);
            a2 = c2[0] + c2[1];
        }
        a2 += __shfl_xor(a2, 1);
        a2 += __shfl_xor(a2, 2);
        if (p == 0) {
            put_y(Yg + (size_t)i * kYG, row, a2, epoch);
            const int nreal = min(b.K, P.ncam - i * b.K) * 6;
            if (row < nreal) P.yF[(size_t)i * b.K * 6 + row] = a2;
            yc[row] = a2;
        }
        __syncthreads();
        // the candidate of camera t of this block (y published above)
        CandAcc ca;
        if (cam) {
            double e[6];
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                e[a] = cand_col(cx[a], yc[6 * t + a], csf[a], cbf[a], ca);
                cand.cand_extr[6 * (size_t)cimg + a] = e[a];
            }
            cand.cand_cp[cimg] = make_campre(e);
        }
        if (t < 16) {
            redc[t][0] = ca.x2;
            redc[t][1] = ca.d2;
            redc[t][2] = ca.gm;
        }
        if (i == 0) {
            // the root: images without camera columns (copied, CamPre rebuilt
            // as cand_kernel does) and the intrinsics (part_f[N])
            for (int f = t; f < P.n_free; f += NT) {
                const int img = P.free_img[f];
                double e[6];
#pragma unroll
                for (int a = 0; a < 6; ++a) {
                    e[a] = cand.extr[6 * (size_t)img + a];
                    cand.cand_extr[6 * (size_t)img + a] = e[a];
                }
                cand.cand_cp[img] = make_campre(e);
            }
            if (t == 0) {
                CandAcc ci;
                // SNAVELY: the 4th double is not a parameter (not moved, not in the norms)
                const int iw = P.iw, na = P.cam_model == SFM_CAM_SNAVELY ? 3 : iw;
                for (int q = 0; q < P.n_intr; ++q) {
                    const int c0 = P.intr_col[q];
                    for (int a = 0; a < iw; ++a) {
                        const double x = cand.intr[iw * (size_t)q + a];
                        const int64_t c = (int64_t)c0 + a;
                        cand.cand_intr[iw * (size_t)q + a] =
                            (c0 >= 0 && a < na) ? cand_col(x, P.yF[c], P.scaleF[c], P.bF[c], ci) : x;
                    }
                }
                P.part_f[3 * (size_t)b.N] = ci.x2;
                P.part_f[3 * (size_t)b.N + 1] = ci.d2;
                P.part_f[3 * (size_t)b.N + 2] = ci.gm;
            }
        }
        __syncthreads();
        if (t == 0) {   // the block's cameras in order
            double r3[3] = {0.0, 0.0, 0.0};
            for (int c = 0; c < b.K; ++c) {
                r3[0] += redc[c][0];
                r3[1] += redc[c][1];
                r3[2] = fmax(r3[2], redc[c][2]);
            }
            for (int k = 0; k < 3; ++k) P.part_f[3 * (size_t)i + k] = r3[k];
        }
    }
    if (FLOW) {   // the last workgroup publishes the verdict (every timeout word drained before its ticket)
        unsigned* counter = reinterpret_cast<unsigned*>(b.fail + 5);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0 &&
            __hip_atomic_fetch_add((gu32*)counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
            P.scal[kScSolveFail] = solve_verdict(b.fail);
            reset_verdict(b);
            __hip_atomic_store((gu32*)counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// the verdict after per-level back substitution launches
__global__ void bcr_verdict_kernel(BcrArgs b, DevProblem P) {
    P.scal[kScSolveFail] = solve_verdict(b.fail);
    reset_verdict(b);
}

}  // namespace

// the bordered arrow: iw * nintr <= 16 columns (one MFMA column tile beside
// the rhs; bcr_corner_part_kernel's 16 lanes, bcr_corner_kernel's 16 x 16)
bool bcr_supported(const DevProblem& P) { return P.D <= kBcrK && P.ncam > 0 && P.iw * P.nintr <= 16; }

void bcr_setup(BcrArgs& b, const DevProblem& P) {
    // K >= D keeps the super-blocks block-tridiagonal; K = 9 for a band of
    // up to 9 camera blocks (C4: a point seen by 10 consecutive cameras):
    // 54 real rows, so the last diagonal tile's factor takes 6 pivots instead
    // of 12 real + 4 padding (diag16_last)
    b.K = std::max(9, P.D);
    b.N = (P.ncam + b.K - 1) / b.K;
    b.nrhs = ((1 + P.iw * P.nintr) + 15) / 16 * 16;   // MFMA column tiles
}

size_t bcr_doubles(const BcrArgs& b) {
    const size_t mm = (size_t)b.N * M * M, mr = (size_t)b.N * M * b.nrhs;
    // A C L(=X) Wl Wr | R Z Y | part | fail (+ counters) | y flags (one word per block)
    return 5 * mm + 3 * mr + 512 * ((size_t)b.N + 1) + 8 + ((size_t)b.N + 1) / 2 + 2;
}

void bcr_bind(BcrArgs& b, double* base) {
    const size_t mm = (size_t)b.N * M * M, mr = (size_t)b.N * M * b.nrhs;
    b.A = base; b.C = b.A + mm; b.L = b.C + mm; b.Wl = b.L + mm; b.Wr = b.Wl + mm;
    b.R = b.Wr + mm; b.Z = b.R + mr; b.Y = b.Z + mr;
    b.part = b.Y + mr; b.fail = b.part + 512 * ((size_t)b.N + 1);
    b.yflag = reinterpret_cast<unsigned*>(b.fail + 8);   // zeroed by the caller once
}

void bcr_solve(const BcrArgs& b, const DevProblem& P, double radius, hipStream_t s, unsigned epoch,
               const BcrCand& cand) {
    if (b.N == 1) {   // no level: the top reads the packed block
        hipLaunchKernelGGL(bcr_pack_kernel, dim3(16 * b.N), dim3(NT), 0, s, b, P, radius);
        SFM_HIP(hipGetLastError());
    }
    const size_t ldr = b.nrhs + 1;
    const size_t lds_odd = (2 * M * LD + 2 * M * M + 2 * M * 17 + 16 * LD + 20) * sizeof(double);
    const size_t lds_even = (2 * M * LD + 2 * M * ldr) * sizeof(double);
    const size_t lds_l = std::max(lds_odd, lds_even);
    const size_t lds_t = (3 * M * LD + 3 * M * ldr + 34) * sizeof(double);
    {   // sized for the largest nrhs (32)
        const size_t cap = 160 * 1024;
        set_dyn_lds((const void*)bcr_level_kernel<false>, cap);
        set_dyn_lds((const void*)bcr_top_kernel, cap);
        set_dyn_lds((const void*)bcr_level_kernel<true>, lds_l);   // (+ the corner's static LDS)
    }
    int s_top = 1;
    for (int stride = 1; stride < b.N; stride *= 2) {
        const int n_odd = (b.N - stride + 2 * stride - 1) / (2 * stride);
        const int n_even = stride > 1 ? (b.N + 2 * stride - 1) / (2 * stride) : 0;
        hipLaunchKernelGGL(bcr_level_kernel<false>, dim3(32 * ((n_odd + n_even + 7) / 8)), dim3(NTL), lds_l, s, b, P,
                           radius, stride, n_odd, 0u);
        SFM_HIP(hipGetLastError());
        s_top = stride * 2;
    }
    // the top, then the corner (one column left for the back substitution) --
    // one launch unless SFM_CTX_BA_SPLIT_BCR (A/B, tests) -- then every
    // back-substitution level in one top-down dataflow launch.  The top runs
    // as a level item (bcr_level_kernel<true>) when it has a neighbour and z_0
    // is one column tile; else as one workgroup (bcr_top_body).
    const bool top_level = b.N >= 2 && b.nrhs == 16;
    if (top_level) {
        hipLaunchKernelGGL(bcr_level_kernel<true>, dim3(b.split ? 4 : 3 + b.N), dim3(NTL), lds_l, s, b, P, radius,
                           s_top, 1, epoch);
        SFM_HIP(hipGetLastError());
        if (b.split) {
            hipLaunchKernelGGL(bcr_corner_kernel, dim3(b.N), dim3(NT), 0, s, b, P, radius);
            SFM_HIP(hipGetLastError());
        }
    } else if (!b.split) {
        set_dyn_lds((const void*)bcr_top_corner_kernel, 156 * 1024);   // (160 KB less the corner's static LDS)
        hipLaunchKernelGGL(bcr_top_corner_kernel, dim3(b.N), dim3(NTL), lds_t, s, b, P, radius, s_top / 2);
        SFM_HIP(hipGetLastError());
    } else {
        hipLaunchKernelGGL(bcr_top_kernel, dim3(1), dim3(NTL), lds_t, s, b, s_top / 2);
        SFM_HIP(hipGetLastError());
        hipLaunchKernelGGL(bcr_corner_kernel, dim3(b.N), dim3(NT), 0, s, b, P, radius);
        SFM_HIP(hipGetLastError());
    }
    int n_back = 1;
    for (int stride = s_top / 2; stride >= 1; stride /= 2) n_back += (b.N - stride + 2 * stride - 1) / (2 * stride);
    if (!b.split) {
        hipLaunchKernelGGL(bcr_back_kernel<true>, dim3(n_back), dim3(NT), 0, s, b, P, s_top, epoch, cand);
        SFM_HIP(hipGetLastError());
    } else {   // SFM_CTX_BA_SPLIT_BCR: one launch per level
        hipLaunchKernelGGL(bcr_back_kernel<false>, dim3(1), dim3(NT), 0, s, b, P, 0, epoch, cand);
        SFM_HIP(hipGetLastError());
        for (int stride = s_top / 2; stride >= 1; stride /= 2) {
            const int n_odd = (b.N - stride + 2 * stride - 1) / (2 * stride);
            hipLaunchKernelGGL(bcr_back_kernel<false>, dim3(n_odd), dim3(NT), 0, s, b, P, stride, epoch, cand);
            SFM_HIP(hipGetLastError());
        }
        hipLaunchKernelGGL(bcr_verdict_kernel, dim3(1), dim3(1), 0, s, b, P);
        SFM_HIP(hipGetLastError());
    }
}


// ===========================================================================
// Dense reduced camera system (RCS) solve: blocked right-looking Cholesky on
// 64x64 fp64 tiles.  Used when the cameras do not form a narrow band (random
// visibility, long tracks, many intrinsics blocks) -- Ceres' SPARSE_SCHUR +
// EIGEN_SPARSE (BundleAdjuster.h:171-173) factors the same matrix.
//   A         lower(S) + D^2 (Ceres' LM diagonal), identity padding; b = rhs --
//             formed by each tile's first reader (pack_elem), no pack pass
//   step k    panel: every workgroup of column k factors A_kk (chol_inv64:
//             L_kk and X_kk = L_kk^-1, MFMA) and forms L_ik = A_ik X_kk';
//             the k-th one stores L_kk, X_kk and y_k = X_kk b_k
//   update k  A_ij -= L_ik L_jk' for k < j <= i (one workgroup per tile, MFMA),
//             b_i -= L_ik y_k (forward substitution, fused); columns go in
//             groups of kDenseW so the trailing tiles are read and written
//             once per group (the update is HBM bound on those tiles)
//   back      x_k = X_kk' y_k, then y_i -= L_ki' x_k for i < k (one launch per k)
// ===========================================================================
namespace {

constexpr int kDM = 64;   // tile
constexpr int kDenseW = 4;   // block columns per trailing update
#ifndef SFM_DENSE_FLOW_MAX_NT
#define SFM_DENSE_FLOW_MAX_NT 100   // (A/B builds only; 29 until round 6)
#endif
constexpr int kDenseFlowMaxNt = SFM_DENSE_FLOW_MAX_NT;   // the dataflow solve up to this many block columns
enum : int { kTaskD = 0, kTaskS = 1, kTaskT = 2, kTaskY = 3, kTaskB = 4 };   // dataflow tasks (dense_flow_plan)

__device__ __forceinline__ void st_wt(double* p, double v) {   // write-through store
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A's first values: lower(S) + D^2 (Ceres' LM diagonal), identity padding,
// 0 above the diagonal, at (a, b).  No pack pass (round 6): each tile's first
// reader -- the first panel, the first group's updates, a dataflow task --
// forms it from the reduce's lower-triangle S (one np^2 write and read less:
// 96 us per dense-S solve)
__device__ __forceinline__ double pack_elem(const DevProblem& P, double radius, int64_t a, int64_t b) {
    if (a < P.nF && b < P.nF) {
        double v = b <= a ? P.Sdense[a * P.nF + b] : 0.0;
        if (a == b) {
            const double lm = sqrt(clampd(P.cnF[a], P.min_diag, P.max_diag) / radius);
            v += lm * lm;
        }
        return v;
    }
    return a == b ? 1.0 : 0.0;
}
__device__ __forceinline__ double pack_rhs(const DevProblem& P, int64_t e) { return e < P.nF ? P.rhs[e] : 0.0; }
// tile (i, j)'s first values into LDS [64][LD] (i >= j)
__device__ __forceinline__ void pack_tile(double* T, const DevProblem& P, double radius, int i, int j) {
    for (int e = threadIdx.x; e < M * M; e += NT)
        T[(e / M) * LD + e % M] = pack_elem(P, radius, (int64_t)i * kDM + e / M, (int64_t)j * kDM + e % M);
}

// column k: workgroup w handles row tile i = k + w
__global__ __launch_bounds__(NT) void dense_panel_kernel(DenseArgs d, DevProblem P, double radius, int k) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* Akk = sm;                 // [64][LD]
    double* Xkk = Akk + M * LD;       // [64][LD]
    double* Aik = Xkk + M * LD;       // [64][LD]
    double* flag = Aik + M * LD;      // [2]
    const int i = k + blockIdx.x;
    const int64_t np = d.np;
    const double* src = d.A + (int64_t)k * kDM * np + (int64_t)k * kDM;
    // A_kk and A_ik in flight together (round 6: one memory latency, not two)
    for (int e = threadIdx.x; e < M * LD; e += NT) Xkk[e] = 0.0;
    if (threadIdx.x == 0) flag[0] = 0.0;
    if (k == 0) {   // the tiles' first reader
        pack_tile(Akk, P, radius, 0, 0);
        if (i > k) pack_tile(Aik, P, radius, i, 0);
    } else if (i > k) {
        load_tiles2(Akk, src, Aik, d.A + (int64_t)i * kDM * np + (int64_t)k * kDM, (int)np);
    } else {
        load_tile<64>(Akk, LD, src, (int)np);
    }
    double* bk = Aik;   // (the diagonal workgroup's b_k, LDS)
    if (i == k && threadIdx.x < M)
        bk[threadIdx.x] = k == 0 ? pack_rhs(P, threadIdx.x) : d.b[(int64_t)k * kDM + threadIdx.x];
    __syncthreads();
    chol_inv64<NT / 64, NoPre, NoPre, NoBg, true>(Akk, Xkk, flag, flag + 1);
    const int wave = threadIdx.x >> 6;
    if (i == k) {
        // X_kk only.  L_kk itself is never read again (the updates and both
        // substitutions use X_kk and the off-diagonal L tiles), and writing it
        // over A_kk raced with this launch's other workgroups, which read A_kk
        // as they start: a workgroup dispatched late -- e.g. behind another
        // stream's kernel holding the CUs -- factored L_kk instead of A_kk.
        // That was the round-3 look-ahead's wrong solves.
        double* xd = d.X + (int64_t)k * kDM * kDM;
        for (int e = threadIdx.x; e < M * M; e += NT) xd[e] = Xkk[(e / M) * LD + e % M];
        // y_k = X_kk b_k (b_k final: every earlier column's update is done;
        // staged in LDS above)
        if (threadIdx.x < M) {
            const int r = threadIdx.x;
            double s = 0.0;
            for (int c = 0; c <= r; ++c) s += Xkk[r * LD + c] * bk[c];
            d.y[(int64_t)k * kDM + r] = s;
        }
        if (threadIdx.x == 0 && flag[0] != 0.0) d.fail[0] = 1.0;
        return;
    }
    // L_ik = A_ik X_kk' (X lower: column c of X' needs m <= c)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int t = wave * 4 + q, ti = t >> 2, tj = t & 3;
        const v4d acc = tile_mm<false, true, false>(zero4(), Aik, LD, 16 * ti, Xkk, LD, 16 * tj, 0, 16 * tj + 16);
        tile_st(d.A + (int64_t)i * kDM * np + (int64_t)k * kDM, (int)np, 16 * ti, 16 * tj, acc);
    }
}

// trailing update from block columns k0 .. k0 + kw - 1: tiles (i, j) with
// j0 <= j <= i (nw > 0: j < j0 + nw only) get A_ij -= sum_kk L_i,kk L_j,kk', the
// accumulator staying in registers across the kw columns (one read and one
// write of A_ij per launch instead of per column; the fp64 MFMA chain is the
// same, so the result is bit-identical); then rhs tiles i > rc get
// b_i -= L_i,rc y_rc (forward substitution, fused).
// Retiled (round 6): the L tiles are staged 32 columns (k) at a time, 34 KB of
// LDS per workgroup instead of 67 KB, so three update workgroups share a CU
// instead of two (waves_per_eu 3: at most 168 VGPRs).  One workgroup
// alternates its MFMAs with waits for the next stage's global loads (L tiles
// from the MALL, a few us); two per CU left the fp64 MFMA pipes ~60 % idle
// at dense-S.  The MFMA sequence of each output tile is unchanged (k ascending
// in 16-deep chunks).  A/B (profiles/r06/d_dense_chain/tiling_ab.txt): dense-S
// 107.9-108.1 (64-column stages, 2 per CU) / 110.0-110.1 (32, 4 per CU) /
// 110.5-110.9 (32, 3 per CU) / 90.6 (16, 6) / 77.8 (16, 8) LM-iters/s.
#ifndef SFM_UPD_KC
#define SFM_UPD_KC 32   // (A/B builds only)
#endif
#ifndef SFM_UPD_WPE
#define SFM_UPD_WPE 3
#endif
constexpr int kUpdKC = SFM_UPD_KC, kUpdLD = kUpdKC + 1;
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(SFM_UPD_WPE, SFM_UPD_WPE)))
void dense_update_kernel(DenseArgs d, DevProblem P, double radius, int k0, int kw, int j0, int n_tiles, int nw,
                         int rc) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* Li = sm;
    double* Lj = sm + M * kUpdLD;
    const int64_t np = d.np;
    const int t = blockIdx.x;
    if (t >= n_tiles) {   // rhs tile i: b_i -= L_i,rc y_rc
        // thread (g, r): columns 16 g .. 16 g + 15 of row r, every load issued
        // first; the four partials summed in a fixed order
        const int i = rc + 1 + (t - n_tiles);
        const int r = threadIdx.x & 63, g = threadIdx.x >> 6;
        const double* L = d.A + ((int64_t)i * kDM + r) * np + (int64_t)rc * kDM + 16 * g;
        const double* yk = d.y + (int64_t)rc * kDM + 16 * g;
        double lv[16], yv[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) { lv[c] = L[c]; yv[c] = yk[c]; }
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < 16; ++c) s = fma(lv[c], yv[c], s);
        sm[g * M + r] = s;
        __syncthreads();
        if (threadIdx.x < M) {
            const int64_t e = (int64_t)i * kDM + r;
            const double b = rc == 0 ? pack_rhs(P, e) : d.b[e];   // (rc = 0: b's first reader)
            d.b[e] = b - (((sm[r] + sm[M + r]) + sm[2 * M + r]) + sm[3 * M + r]);
        }
        return;
    }
    int i, j;
    if (nw > 0) {   // the nw block columns from j0, rectangle of rows j0 .. nt - 1
        const int rows = d.nt - j0;
        i = j0 + t % rows;
        j = j0 + t / rows;
        if (i < j) return;   // above the diagonal: whole workgroup
    } else {   // t -> (i, j) over the lower triangle of the trailing tile grid
        int a = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
        while ((a + 1) * (a + 2) / 2 <= t) ++a;
        while (a * (a + 1) / 2 > t) --a;
        i = j0 + a;
        j = j0 + (t - a * (a + 1) / 2);
    }
    double* C = d.A + (int64_t)i * kDM * np + (int64_t)j * kDM;
    const int wave = threadIdx.x >> 6;
    const double* Lb = i != j ? Lj : Li;
    v4d acc[4];
    const bool first = k0 == 0;   // the first group's updates are the tiles' first readers
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int tt = wave * 4 + q, ti = tt >> 2, tj = tt & 3;
        if (i == j && tj > ti) {
            acc[q] = zero4();
        } else if (first) {
            const int lane = threadIdx.x & 63, kk = lane >> 4;
#pragma unroll
            for (int r = 0; r < 4; ++r)
                acc[q][r] = pack_elem(P, radius, (int64_t)i * kDM + 16 * ti + kk + 4 * r,
                                      (int64_t)j * kDM + 16 * tj + (lane & 15));
        } else {
            acc[q] = tile_ld(C, (int)np, 16 * ti, 16 * tj);
        }
    }
    // stage st = (column kk, half h): the L_ik / L_jk columns 32 h .. 32 h + 31
    // of column kk; the next stage's are fetched into registers while this
    // stage's MFMAs run
    TileFetch<kUpdKC, M, NT> fi, fj;
    constexpr int kSt = M / kUpdKC;   // stages per column
    auto fetch = [&](int st) {
        const int64_t off = (int64_t)(k0 + st / kSt) * kDM + kUpdKC * (st % kSt);
        fi.fetch(d.A + (int64_t)i * kDM * np + off, (int)np);
        if (i != j) fj.fetch(d.A + (int64_t)j * kDM * np + off, (int)np);
    };
    const int n_st = kSt * kw;
    fetch(0);
    for (int st = 0; st < n_st; ++st) {
        if (st > 0) __syncthreads();   // the previous stage's tiles are consumed
        fi.put(Li, kUpdLD);
        if (i != j) fj.put(Lj, kUpdLD);
        __syncthreads();
        if (st + 1 < n_st) fetch(st + 1);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int tt = wave * 4 + q, ti = tt >> 2, tj = tt & 3;
            if (i == j && tj > ti) continue;   // the diagonal tile's lower half (and its diagonal sub-tiles)
            acc[q] = tile_mm<false, true, true>(acc[q], Li, kUpdLD, 16 * ti, Lb, kUpdLD, 16 * tj, 0, kUpdKC);
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int tt = wave * 4 + q, ti = tt >> 2, tj = tt & 3;
        if (i == j && tj > ti && !first) continue;   // (first: the upper 16x16 tiles go out as zeros)
        tile_st(C, (int)np, 16 * ti, 16 * tj, acc[q]);
    }
}

// back substitution L' x = y, right-looking by block column, one launch per
// k (descending): every workgroup forms x_k = X_kk' y_k (y_k is final: the
// launches for j > k have subtracted their L_jk' x_j), then workgroup i < k
// applies y_i -= L_ki' x_k from row block k (contiguous rows).  The k = 0
// launch also publishes x to yF.
__global__ __launch_bounds__(NT) void dense_back_kernel(DenseArgs d, DevProblem P, int k) {
    __shared__ double Xs[M * (M + 1)], yk[M], xk[M], part[4][M];
    const int64_t np = d.np;
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    {   // X_kk and y_k into LDS: all loads in flight at once
        const double* X = d.X + (int64_t)k * kDM * kDM;
        double v[M / 4];
#pragma unroll
        for (int q = 0; q < M / 4; ++q) v[q] = X[(4 * q + g) * M + c];
#pragma unroll
        for (int q = 0; q < M / 4; ++q) Xs[(4 * q + g) * (M + 1) + c] = v[q];
        if (threadIdx.x < M) yk[c] = d.y[(int64_t)k * kDM + c];
    }
    __syncthreads();
    if (threadIdx.x < M) {   // x_k = X_kk' y_k: X lower, so rows m >= c
        double v = 0.0;
        for (int mm = c; mm < M; ++mm) v += Xs[mm * (M + 1) + c] * yk[mm];
        xk[c] = v;
        if (blockIdx.x == 0) d.x[(int64_t)k * kDM + c] = v;
    }
    __syncthreads();
    if (k == 0) {
        for (int64_t e = threadIdx.x; e < P.nF; e += NT) P.yF[e] = e < M ? xk[e] : d.x[e];
        if (threadIdx.x == 0) {
            P.scal[kScSolveFail] = solve_verdict(d.fail);
            d.fail[0] = 0.0;   // cleared for the next solve (no pack pass clears them)
            d.fail[1] = 0.0;
        }
        return;
    }
    const int i = blockIdx.x;   // < k
    const double* L = d.A + (int64_t)k * kDM * np + (int64_t)i * kDM + c;
    double lv[M / 4];
#pragma unroll
    for (int q = 0; q < M / 4; ++q) lv[q] = L[(int64_t)(4 * q + g) * np];
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < M / 4; ++q) s += lv[q] * xk[4 * q + g];
    part[g][c] = s;
    __syncthreads();
    if (threadIdx.x < M) d.y[(int64_t)i * kDM + c] -= ((part[0][c] + part[1][c]) + part[2][c]) + part[3][c];
}

// back substitution, every block column in one launch (dataflow): workgroup
// w takes block k = nt - 1 - w, accumulates y_k - sum_{j>k} L_jk' x_j as the
// x_j arrive (j descending, each L_jk slice loaded before its wait), then
// x_k = X_kk' (...) and publishes x_k.  Workgroup k waits only for workgroups
// of lower index (in-order dispatch), one workgroup per CU (the dynamic LDS
// below is sized for that), every workgroup resident (nt <= the CU count,
// checked by the caller), and every spin bounded (a timeout marks the solve
// failed: SFM_ERR_DEVICE).
// Round 6: two columns of lookahead and tagged x granules.  The substitution's
// chain is x_k+1 -> x_k (4.2 us per column at dense-S: the flag poll, a
// 64-long dependent X' v loop, the drain, the flag).  Now
//   x_k = r_k - M1 x_k+1 - M2 x_k+2,   M1 = X_k' L_k+1,k',  M2 = X_k' L_k+2,k',
//   r_k = X_k' (y_k - sum_{j > k+2} L_jk' x_j)
// with M1 / M2 formed at the start (MFMA) and held in registers, r_k ready
// once x_k+3 is in, so the arrival of x_k+1 costs a 64 x 64 matrix-vector
// product from registers; x_k goes out as 128 tagged granules (put_y / get_y:
// the data is the flag -- no drain, no flag round trip).
__global__ __launch_bounds__(NT) void dense_back_all_kernel(DenseArgs d, DevProblem P, unsigned epoch) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* Xs = sm;                  // [64][LD] X_k
    double* Lt = Xs + M * LD;         // [64][LD] L_k+1,k, then L_k+2,k
    double* Mt = Lt + M * LD;         // [64][LD] M1, then M2
    double* xs = Mt + M * LD;         // [2][64] x_j, double buffered
    double* part = xs + 2 * M;        // [4][64]
    double* v = part + 4 * M;         // [64]
    double* part2 = v + M;            // [4][64]
    double* part3 = part2 + 4 * M;    // [4][64]
    const int nt = d.nt, k = nt - 1 - (int)blockIdx.x;
    const int64_t np = d.np;
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6, wave = g;
    auto tL = [&](int j) { return d.A + (int64_t)j * kDM * np + (int64_t)k * kDM; };   // L_jk
    load_tile<64>(Xs, LD, d.X + (int64_t)k * kDM * kDM, M);
    double m1[16], m2[16];
    auto form = [&](int j, double (&mr)[16]) {   // mr = row c, columns 16 g .. of X_k' L_jk'
        load_tile<64>(Lt, LD, tL(j), (int)np);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q)
            tile_st(Mt, LD, 16 * wave, 16 * q,
                    tile_mm<true, true, false>(zero4(), Xs, LD, 16 * wave, Lt, LD, 16 * q, 16 * wave, M));
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 16; ++q) mr[q] = Mt[c * LD + 16 * g + q];
        __syncthreads();   // (Lt / Mt reused)
    };
    if (k + 1 < nt) form(k + 1, m1);
    if (k + 2 < nt) form(k + 2, m2);
    __syncthreads();
    // r_k: the x_j of j > k + 2 as they arrive (each L_jk slice fetched first)
    double s = 0.0;
    int buf = 0;
    for (int j = nt - 1; j > k + 2; --j) {
        const double* L = tL(j) + c;
        double lr[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) lr[q] = L[(int64_t)(4 * q + g) * np];
        double* xb = xs + M * buf;
        if (wave == 0) get_y(d.xg + (int64_t)j * kYG, nullptr, xb, nullptr, epoch, d.fail);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 16; ++q) s = fma(lr[q], xb[4 * q + g], s);
        buf ^= 1;
    }
    part[g * M + c] = s;
    __syncthreads();
    if (threadIdx.x < M)
        v[c] = d.y[(int64_t)k * kDM + c] - (((part[c] + part[M + c]) + part[2 * M + c]) + part[3 * M + c]);
    __syncthreads();
    // r_k = X_k' v (X lower: rows m >= c), rows 16 g .. 16 g + 15 per thread
    double u = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int m = 16 * g + q;
        if (m >= c) u = fma(Xs[m * LD + c], v[m], u);
    }
    part2[g * M + c] = u;
    __syncthreads();
    double xv = ((part2[c] + part2[M + c]) + part2[2 * M + c]) + part2[3 * M + c];
    if (k + 1 < nt) {
        double w = 0.0;
        if (k + 2 < nt) {   // x_k+2 first (it arrives first), then x_k+1
            double* xb = xs + M * buf;
            if (wave == 0) get_y(d.xg + (int64_t)(k + 2) * kYG, nullptr, xb, nullptr, epoch, d.fail);
            __syncthreads();
#pragma unroll
            for (int q = 0; q < 16; ++q) w = fma(m2[q], xb[16 * g + q], w);
            buf ^= 1;
        }
        double* xb = xs + M * buf;
        if (wave == 0) get_y(d.xg + (int64_t)(k + 1) * kYG, nullptr, xb, nullptr, epoch, d.fail);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 16; ++q) w = fma(m1[q], xb[16 * g + q], w);
        part3[g * M + c] = w;
        __syncthreads();
        xv -= ((part3[c] + part3[M + c]) + part3[2 * M + c]) + part3[3 * M + c];
    }
    if (threadIdx.x < M) {
        put_y(d.xg + (int64_t)k * kYG, c, xv, epoch);
        const int64_t e = (int64_t)k * kDM + c;
        if (e < P.nF) P.yF[e] = xv;
    }
    // block 0 finishes last (it waits for every other x): the solve's verdict
    // (the failure words come from the earlier launches), then the words
    // cleared for the next solve (no pack pass clears them)
    if (k == 0 && threadIdx.x == 0) {
        P.scal[kScSolveFail] = solve_verdict(d.fail);
        st_wt(d.fail, 0.0);
        st_wt(d.fail + 1, 0.0);
    }
}

// ---- the whole factorisation + both substitutions in one dataflow launch ----
// For dense systems up to kDenseFlowMaxNt block columns (the C5 loop's, nt <=
// 29; RADIAL3 per camera, 38; dense-S, 94) the panel / update launch chain is
// latency bound (a 64-pivot factor per column plus two launches).  Here workgroup 0 runs the diagonal chain -- for k: L_k,k-1 =
// A~_k,k-1 X_k-1', A_kk -= L_k,k-1 L_k,k-1', factor + invert A_kk -- and every
// other workgroup owns one task, left-looking:
//   D(i)     A~_ii    = A_ii    - sum_{m < i-1} L_im L_im'       (for the chain)
//   S(i)     A~_i,i-1 = A_i,i-1 - sum_{m < i-1} L_im L_i-1,m'    (for the chain)
//   T(i, j)  L_ij = (A_ij - sum_{m < j} L_im L_jm') X_j'         (i >= j + 2)
//   Y(j)     y_j = X_j (b_j - sum_{m < j} L_jm y_m)
//   B(k)     x_k = X_k' (y_k - sum_{i > k} L_ik' x_i)
// Each accumulates its terms as their inputs are published, in m order.
// Hand-offs: payload stored write-through (agent-scope stores), every storing
// wave drains, the workgroup meets, one lane stores the flag; consumers poll
// relaxed, acquire once per run of ready inputs, then read plainly
// (cdna_hip_programming.md Guideline 16).  Every workgroup is resident (one
// per CU, at most n_cu: the caller) and the task workers take tasks round
// robin in an order where every input comes from a lower task or the chain,
// so every wait ends; spins are bounded (a timeout fails the solve).
constexpr int kDfLds = 4 * M * LD + 32;   // doubles: four tiles + small state

__device__ __forceinline__ void tile_st_wt(double* C, int ldc, int r0, int c0, v4d v) {
    const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) st_wt(C + (r0 + kk + 4 * r) * (int64_t)ldc + c0 + i, v[r]);
}
// publish: every storing wave drains, the workgroup meets, one lane flags
__device__ __forceinline__ void df_publish(unsigned* flag, unsigned epoch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void df_publish2(unsigned* f1, unsigned* f2, unsigned epoch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(f1, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(f2, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// wait until fa[m * sa] (and fb[m * sb], if given) hold epoch for m = m0 and
// return the end m' <= m1 of the run of ready m from m0 (one acquire for all);
// every thread gets it (the workgroup meets)
__device__ __forceinline__ int df_wait_run(const unsigned* fa, int sa, const unsigned* fb, int sb, int m0, int m1,
                                           unsigned epoch, double* fail, int* sh) {
    if (threadIdx.x == 0) {
        auto ready = [&](int m) {   // (both flags loaded together: one round trip)
            const unsigned a = __hip_atomic_load(fa + (int64_t)m * sa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned b =
                fb ? __hip_atomic_load(fb + (int64_t)m * sb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : epoch;
            return (a == epoch) & (b == epoch);
        };
        unsigned spins = 0;
        while (!ready(m0)) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 22)) {
                __hip_atomic_store(fail + 1, 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // timeout
                break;
            }
        }
        int m = m0 + 1;
        while (m < m1 && ready(m)) ++m;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *sh = m;
    }
    __syncthreads();
    return *sh;
}
// wait until the flags of term m[0] hold epoch (fa + m * sa, and fb + m * sb
// if given), then count how many of the terms m[0 .. n) are ready from the
// first on (at least 1; one acquire for all); every thread gets the count
__device__ __forceinline__ int df_wait_batch(const unsigned* fa, int sa, const unsigned* fb, int sb, const int (&mb)[4],
                                             int n, unsigned epoch, double* fail, int* sh) {
    if (threadIdx.x == 0) {
        // every flag of the batch loaded at once (one round trip, not one per
        // term and flag), then term 0's re-polled until it is set
        unsigned va[4], vb[4];
        auto fetch = [&](int q1) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (q < q1) {
                    const int m = q == 0 ? mb[0] : q == 1 ? mb[1] : q == 2 ? mb[2] : mb[3];
                    va[q] = __hip_atomic_load(fa + (int64_t)m * sa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    vb[q] = fb ? __hip_atomic_load(fb + (int64_t)m * sb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : epoch;
                }
        };
        fetch(n);
        unsigned spins = 0;
        while (va[0] != epoch || vb[0] != epoch) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 22)) {
                __hip_atomic_store(fail + 1, 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // timeout
                break;
            }
            fetch(1);
        }
        int cnt = 1;
        bool run = true;
#pragma unroll
        for (int q = 1; q < 4; ++q) {
            run = run && q < n && va[q] == epoch && vb[q] == epoch;
            cnt += run ? 1 : 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *sh = cnt;
    }
    __syncthreads();
    return *sh;
}

// tile (pi, pj) of S in the natural tile order (pi, pj: physical tiles of
// a permuted pair) straight from the reduce's lower-triangle S, with the LM
// diagonal D^2 and identity padding -- pack_elem's values --
// into LDS [64][LD].  A tile above the diagonal (pi < pj) is the transpose
// of the stored lower one.  (The dataflow solve has no pack pass: round 6.)
__device__ __forceinline__ void df_load_a(double* T, const DevProblem& P, double radius, int pi, int pj) {
    const int64_t nF = P.nF, R0 = (int64_t)pi * kDM, C0 = (int64_t)pj * kDM;
    for (int e = threadIdx.x; e < M * M; e += NT) {
        double v = 0.0;
        int r, c;
        if (pi >= pj) {   // source rows, c fastest
            r = e / M;
            c = e % M;
            const int64_t a = R0 + r, b = C0 + c;
            if (a < nF && b < nF) {
                if (pi > pj || c <= r) v = P.Sdense[a * nF + b];
                if (pi == pj && r == c) {
                    const double lm = sqrt(clampd(P.cnF[a], P.min_diag, P.max_diag) / radius);
                    v += lm * lm;
                }
            } else if (pi == pj && r == c) {
                v = 1.0;
            }
        } else {          // transposed: (r, c) = S[C0 + c][R0 + r], r fastest
            c = e / M;
            r = e % M;
            const int64_t a = C0 + c, b = R0 + r;
            if (a < nF && b < nF) v = P.Sdense[a * nF + b];
        }
        T[r * LD + c] = v;
    }
}

__global__ __launch_bounds__(NT) void dense_flow_kernel(DenseArgs d, DevProblem P, double radius, unsigned epoch) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* T1 = sm;
    double* T2 = sm + M * LD;
    double* T3 = T2 + M * LD;      // the chain's diagonal tile; a task's first A tile
    double* T4 = T3 + M * LD;      // a D / S task's X_m (an L_im formed in place)
    double* bad = T4 + M * LD;     // [2]
    double* col = bad + 2;         // [16] (diag16)
    int* sh = reinterpret_cast<int*>(col + 16);
    const int nt = d.nt, wave = threadIdx.x >> 6;
    const int64_t np = d.np;
    unsigned* fL = d.fflag;                 // [nt][nt]: L_ij final (i > j), X_j final (i == j)
    unsigned* fR = d.fflag + nt * nt;       // [nt][nt]: A~_kk (D), A~_kp (S) ready for the chain
    unsigned* fy = d.fflag + 2 * nt * nt;   // [nt]
    // the host's schedule (dense_flow_plan): permuted column k is natural tile perm[k]
    const int32_t* perm = d.meta;
    const int32_t* prevc = d.meta + nt;      // the chain's previous column (-1: none)
    const int32_t* info = d.meta + 2 * nt;   // 1 linked to prevc, 2 D(k) task, 4 S(k) task
    const int32_t* lav = d.meta + 3 * nt;    // the back substitution's lookahead row
    const int32_t* tasks = d.meta + 6 * nt + 2;
    // tile pattern of L: bit 0 nonzero, bit 1 formed by a T task with no
    // terms (L_ij = A_ij X_j', which a D / S task forms itself: dense_flow_plan)
    const unsigned char* nzb = reinterpret_cast<const unsigned char*>(tasks + d.ntask);
    auto nz = [&](int i, int j) { return nzb[i * nt + j] != 0; };
    auto tA = [&](int i, int j) { return d.A + (int64_t)perm[i] * kDM * np + (int64_t)perm[j] * kDM; };
    // ---------------- the diagonal chains ----------------
    if ((int)blockIdx.x < d.nch) {
        const int32_t* clist = d.meta + (4 + blockIdx.x) * nt;
        const int clen = d.meta[6 * nt + blockIdx.x];
        unsigned long long ts[7] = {0, 0, 0, 0, 0, 0, 0}, tp = 0;
        const bool stm = d.stamps != nullptr;
        auto mark = [&](int ph) {
            if (stm) {
                const unsigned long long tn = stamp();
                ts[ph] += tn - tp;
                tp = tn;
            }
        };
        // X_k (in T2) to global, write-through; the factor's verdict with it
        auto x_out = [&](int k) {
            double* xd = d.X + (int64_t)k * kDM * kDM;
            for (int e = threadIdx.x; e < M * M; e += NT) st_wt(xd + e, T2[(e / M) * LD + e % M]);
            if (threadIdx.x == 0 && bad[0] != 0.0) st_wt(d.fail, 1.0);
        };
        if (stm) tp = stamp();
        const unsigned long long rt0 = stm ? __builtin_amdgcn_s_memrealtime() : 0;
        for (int q = 0; q < clen; ++q) {
            const int k = clist[q], p = prevc[k], inf = info[k];
            const bool hd = (inf & 2) != 0, hs = (inf & 4) != 0;
            if (inf & 1) {
                // linked: T2 holds X_p.  A~_kp to T1 and A~_kk to T3, loaded together
                if (hs || hd)
                    df_wait_run(hs ? fR + k * nt + p : fR + k * nt + k, 0, (hs && hd) ? fR + k * nt + k : nullptr, 0, 0,
                                1, epoch, d.fail, sh);   // S(k), D(k)
                mark(0);
                if (hs && hd) {
                    load_tiles2(T1, tA(k, p), T3, tA(k, k), (int)np);
                } else {
                    if (hs) load_tile<64>(T1, LD, tA(k, p), (int)np);
                    else df_load_a(T1, P, radius, perm[k], perm[p]);
                    if (hd) load_tile<64>(T3, LD, tA(k, k), (int)np);
                    else df_load_a(T3, P, radius, perm[k], perm[k]);
                }
                __syncthreads();
                // L_kp = A~_kp X_p'
                v4d acc[4];
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    acc[c] = tile_mm<false, true, false>(zero4(), T1, LD, 16 * wave, T2, LD, 16 * c, 0, 16 * c + 16);
#pragma unroll
                for (int c = 0; c < 4; ++c) tile_st_wt(tA(k, p), (int)np, 16 * wave, 16 * c, acc[c]);
                // X_p goes out with L_kp; their drain and flags come after the
                // diagonal update below, so the stores complete meanwhile
                x_out(p);
                __syncthreads();   // T1 and T2 are read
#pragma unroll
                for (int c = 0; c < 4; ++c) tile_st(T1, LD, 16 * wave, 16 * c, acc[c]);
                for (int e = threadIdx.x; e < M * LD; e += NT) T2[e] = 0.0;
                mark(1);
                __syncthreads();
                // A~_kk -= L L': the 10 lower 16x16 tiles round robin over the waves
                for (int c = wave; c < 10; c += NT / 64) {
                    const int ti = c < 1 ? 0 : c < 3 ? 1 : c < 6 ? 2 : 3;
                    const int tj = c - ti * (ti + 1) / 2;
                    const v4d a = tile_ld(T3, LD, 16 * ti, 16 * tj);
                    tile_st(T3, LD, 16 * ti, 16 * tj, tile_mm<false, true, true>(a, T1, LD, 16 * ti, T1, LD, 16 * tj, 0, M));
                }
                df_publish2(fL + k * nt + p, fL + p * nt + p, epoch);   // L_kp and X_p
                mark(2);
            } else {
                if (hd) {
                    df_wait_run(fR + k * nt + k, 0, nullptr, 0, 0, 1, epoch, d.fail, sh);   // D(k)
                    load_tile<64>(T3, LD, tA(k, k), (int)np);
                } else {
                    df_load_a(T3, P, radius, perm[k], perm[k]);
                }
                for (int e = threadIdx.x; e < M * LD; e += NT) T2[e] = 0.0;
            }
            if (threadIdx.x == 0) bad[0] = 0.0;
            __syncthreads();
            mark(3);
            chol_inv64<NT / 64, NoPre, NoPre, NoBg, true>(T3, T2, bad, col, stm ? d.stamps + 8 : nullptr);
            mark(4);
            // X_k goes out now unless the chain's next column is linked to k
            // (then with L_next,k)
            const int nx = q + 1 < clen ? clist[q + 1] : -1;
            if (nx < 0 || !(info[nx] & 1)) {
                x_out(k);
                df_publish(fL + k * nt + k, epoch);
                mark(5);
            }
        }
        if (stm && threadIdx.x == 0) {
            // (diagnostic) the chains' end in real time (100 MHz, one clock for
            // every CU): the last back-substitution task adds its own end minus
            // the later chain's to slot 25
            const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
            atomicMax(d.stamps + 26, rt1);
            if (blockIdx.x == 0) {
                atomicAdd(d.stamps + 24, rt1 - rt0);
                atomicAdd(d.stamps + 27, 1ull);
            }
            for (int c = 0; c < 6; ++c) atomicAdd(d.stamps + c, ts[c]);
            atomicAdd(d.stamps + 6, (unsigned long long)clen);
        }
        return;
    }
    // ---------------- tasks: in the host's order, round robin over the workers ----------------
    // (every task waits only on earlier tasks and on chain steps that wait
    // only on earlier tasks, so the earliest unfinished one can always run:
    // its worker has finished the ones before it)
    auto task = [&](int t) {
        const int code = tasks[t], kind = code >> 24, i = (code >> 12) & 0xfff, j = code & 0xfff;
        if (kind <= kTaskT) {
            // D(i): A~_ii = A_ii - sum L_im L_im' (m < i, not the chain's own
            // m = prevc[i]); S(i): A~_ij = A_ij - sum L_im L_jm' (m < j = prevc[i]);
            // T(i, j): L_ij = (A_ij - sum_{m < j} L_im L_jm') X_j'.  Nonzero m only.
            const bool diag = kind == kTaskD;
            const int excl = (diag && (info[i] & 1)) ? prevc[i] : -1, mend = diag ? i : j;
            df_load_a(T3, P, radius, perm[i], perm[j]);
            __syncthreads();
            v4d acc[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[c] = (diag && c > wave) ? zero4() : tile_ld(T3, LD, 16 * wave, 16 * c);
            __syncthreads();   // (T3 is reused below)
            // the terms in m order; runs of ready terms in batches (up to four
            // L_im of a D task, two L_im / L_jm pairs otherwise) loaded with
            // one memory latency (round 6: the dense-S solve is bound by its
            // task workers' throughput); the same products in the same order
            auto term_at = [&](int m) {   // the next term from m on (mend: none)
                for (; m < mend; ++m)
                    if (m != excl && nzb[i * nt + m] && (diag || nz(j, m))) break;
                return m;
            };
            const int bmax = diag ? 4 : 2;
            for (int m = term_at(0); m < mend;) {
                const int zi = nzb[i * nt + m];
                if (!((zi & 2) && kind != kTaskT)) {
                    // (registers, no dynamic indexing: the batch's terms)
                    int mb[4] = {m, m, m, m}, nb = 1, q = term_at(m + 1);
#pragma unroll
                    for (int t = 1; t < 4; ++t)
                        if (nb == t && t < bmax && q < mend && !((nzb[i * nt + q] & 2) && kind != kTaskT)) {
                            mb[t] = q;
                            nb = t + 1;
                            q = term_at(q + 1);
                        }
                    const int nr = df_wait_batch(fL + i * nt, 1, diag ? nullptr : fL + j * nt, 1, mb, nb, epoch, d.fail, sh);
                    if (diag)
                        load_tiles4(nr, T1, tA(i, mb[0]), T2, tA(i, mb[1]), T3, tA(i, mb[2]), T4, tA(i, mb[3]), (int)np);
                    else
                        load_tiles4(2 * nr, T1, tA(i, mb[0]), T2, tA(j, mb[0]), T3, tA(i, mb[1]), T4, tA(j, mb[1]),
                                    (int)np);
                    __syncthreads();
                    double* const Tb[4] = {T1, T2, T3, T4};
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        if (b >= nr) break;
                        const double* La = diag ? Tb[b] : Tb[2 * (b & 1)];
                        const double* Lb = diag ? Tb[b] : Tb[2 * (b & 1) + 1];
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            if (diag && c > wave) continue;
                            acc[c] = tile_mm<false, true, true>(acc[c], La, LD, 16 * wave, Lb, LD, 16 * c, 0, M);
                        }
                    }
                    __syncthreads();
                    m = nr == nb ? q : nr == 1 ? mb[1] : nr == 2 ? mb[2] : mb[3];
                    continue;
                }
                {
                    // L_im = A_im X_m' formed here, from the values T(i, m) uses
                    // (same products, same bits): the chain's inputs wait on
                    // X_m instead of on T(i, m)'s hand-off (round 6)
                    df_load_a(T3, P, radius, perm[i], perm[m]);
                    df_wait_run(fL + m * nt + m, 0, diag ? nullptr : fL + j * nt + m, 0, 0, 1, epoch, d.fail, sh);
                    load_tile<64>(T4, LD, d.X + (int64_t)m * kDM * kDM, M);
                    if (!diag) load_tile<64>(T2, LD, tA(j, m), (int)np);
                    __syncthreads();
                    v4d l[4];
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        l[c] = tile_mm<false, true, false>(zero4(), T3, LD, 16 * wave, T4, LD, 16 * c, 0, 16 * c + 16);
#pragma unroll
                    for (int c = 0; c < 4; ++c) tile_st(T1, LD, 16 * wave, 16 * c, l[c]);
                }
                __syncthreads();
                const double* Lb = diag ? T1 : T2;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    if (diag && c > wave) continue;
                    acc[c] = tile_mm<false, true, true>(acc[c], T1, LD, 16 * wave, Lb, LD, 16 * c, 0, M);
                }
                __syncthreads();
                m = term_at(m + 1);
            }
            if (kind != kTaskT) {
                // (the diagonal tile's upper 16x16 tiles go out as zeros: the
                // chain loads the whole tile)
#pragma unroll
                for (int c = 0; c < 4; ++c) tile_st_wt(tA(i, j), (int)np, 16 * wave, 16 * c, acc[c]);
                df_publish(fR + i * nt + j, epoch);
                return;
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) tile_st(T1, LD, 16 * wave, 16 * c, acc[c]);
            df_wait_run(fL + j * nt + j, 0, nullptr, 0, 0, 1, epoch, d.fail, sh);   // X_j
            load_tile<64>(T2, LD, d.X + (int64_t)j * kDM * kDM, M);
            __syncthreads();
#pragma unroll
            for (int c = 0; c < 4; ++c)
                acc[c] = tile_mm<false, true, false>(zero4(), T1, LD, 16 * wave, T2, LD, 16 * c, 0, 16 * c + 16);
#pragma unroll
            for (int c = 0; c < 4; ++c) tile_st_wt(tA(i, j), (int)np, 16 * wave, 16 * c, acc[c]);
            df_publish(fL + i * nt + j, epoch);
            return;
        }
        if (kind == kTaskY) {
            // Y(j): y_j = X_j (b_j - sum L_jm y_m); thread (g, r) sums columns
            // 16 g .. 16 g + 15 of row r of every nonzero L_jm
            const int r = threadIdx.x & 63, g = threadIdx.x >> 6;
            double s = 0.0;
            for (int m = 0; m < j; ++m) {
                if (!nz(j, m)) continue;
                df_wait_run(fL + j * nt + m, 0, fy + m, 0, 0, 1, epoch, d.fail, sh);
                const double* L = tA(j, m) + (int64_t)r * np + 16 * g;
                const double* y = d.y + (int64_t)m * kDM + 16 * g;
#pragma unroll
                for (int c = 0; c < 16; ++c) s = fma(L[c], y[c], s);
            }
            double* part = T1;   // [4][64]
            double* v = T1 + 4 * M;
            double* part2 = T1 + 5 * M;   // [4][64]
            part[g * M + r] = s;
            df_wait_run(fL + j * nt + j, 0, nullptr, 0, 0, 1, epoch, d.fail, sh);   // X_j (the workgroup meets)
            load_tile<64>(T2, LD, d.X + (int64_t)j * kDM * kDM, M);
            if (threadIdx.x < M) {
                const int64_t e = (int64_t)perm[j] * kDM + r;
                v[r] = (e < P.nF ? P.rhs[e] : 0.0) - (((part[r] + part[M + r]) + part[2 * M + r]) + part[3 * M + r]);
            }
            __syncthreads();
            // y_j = X_j v (X lower: columns c <= r), columns 16 g .. 16 g + 15
            // per thread from LDS, the four partials summed in a fixed order
            double u = 0.0;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int c = 16 * g + q;
                if (c <= r) u = fma(T2[r * LD + c], v[c], u);
            }
            part2[g * M + r] = u;
            __syncthreads();
            if (threadIdx.x < M)
                st_wt(d.y + (int64_t)j * kDM + r, ((part2[r] + part2[M + r]) + part2[2 * M + r]) + part2[3 * M + r]);
            df_publish(fy + j, epoch);
            return;
        }
        // B(k): x_k = X_k' (y_k - sum_{i > k} L_ik' x_i) over the nonzero L_ik,
        // with one row of lookahead (round 6), la = the first such i (its x
        // arrives last):
        //   x_k = r_k - M_k x_la,  r_k = X_k' (y_k - sum_{i > k, i != la} L_ik' x_i),
        //   M_k = X_k' L_la,k'  (formed while the substitution is still far)
        // so the arrival of x_la costs one 64 x 64 matrix-vector product from
        // registers.  x goes out as tagged granules (put_y / get_y: the data is
        // the flag, no drain, no flag round trip); every L_ik slice is fetched
        // before its x_i is awaited.
        const int k = i, la = lav[k];
        const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
        // X_k and every nonzero L_ik (i > k): final when the factorisation passes k
        df_wait_run(fL + k * nt + k, 0, nullptr, 0, 0, 1, epoch, d.fail, sh);
        for (int r = k + 1; r < nt; ++r)
            if (nz(r, k)) df_wait_run(fL + r * nt + k, 0, nullptr, 0, 0, 1, epoch, d.fail, sh);
        load_tile<64>(T2, LD, d.X + (int64_t)k * kDM * kDM, M);
        if (la >= 0) load_tile<64>(T1, LD, tA(la, k), (int)np);
        __syncthreads();
        double mreg[16];
        if (la >= 0) {
            // M_k = X_k' L_la,k' (X lower: X[kk][m] = 0 for kk < m)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                tile_st(T3, LD, 16 * wave, 16 * q,
                        tile_mm<true, true, false>(zero4(), T2, LD, 16 * wave, T1, LD, 16 * q, 16 * wave, M));
            __syncthreads();
#pragma unroll
            for (int q = 0; q < 16; ++q) mreg[q] = T3[c * LD + 16 * g + q];
        }
        double* xs = T1;               // [2][64] x_i, double buffered
        double* part = T1 + 2 * M;     // [4][64]
        double* v = T1 + 6 * M;        // [64]
        double* part2 = T1 + 7 * M;    // [4][64]
        double* part3 = T1 + 11 * M;   // [4][64]
        __syncthreads();               // (T1's L tile is read)
        double s = 0.0;
        int buf = 0;
        for (int r = nt - 1; r > k; --r) {   // x_r arrive in this order
            if (r == la || !nz(r, k)) continue;
            const double* L = tA(r, k) + c;
            double lr[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) lr[q] = L[(int64_t)(4 * q + g) * np];
            double* xb = xs + M * buf;
            if (wave == 0) get_y(d.xg + (int64_t)r * kYG, nullptr, xb, nullptr, epoch, d.fail);
            __syncthreads();
#pragma unroll
            for (int q = 0; q < 16; ++q) s = fma(lr[q], xb[4 * q + g], s);
            buf ^= 1;
        }
        part[g * M + c] = s;
        df_wait_run(fy + k, 0, nullptr, 0, 0, 1, epoch, d.fail, sh);   // y_k (the workgroup meets)
        if (threadIdx.x < M)
            v[c] = d.y[(int64_t)k * kDM + c] - (((part[c] + part[M + c]) + part[2 * M + c]) + part[3 * M + c]);
        __syncthreads();
        // r_k = X_k' v (X lower: rows m >= c), rows 16 g .. 16 g + 15 per thread
        double u = 0.0;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int m = 16 * g + q;
            if (m >= c) u = fma(T2[m * LD + c], v[m], u);
        }
        part2[g * M + c] = u;
        __syncthreads();
        double xv = ((part2[c] + part2[M + c]) + part2[2 * M + c]) + part2[3 * M + c];
        if (la >= 0) {
            double* xb = xs + M * buf;
            if (wave == 0) get_y(d.xg + (int64_t)la * kYG, nullptr, xb, nullptr, epoch, d.fail);
            __syncthreads();
            double w = 0.0;
#pragma unroll
            for (int q = 0; q < 16; ++q) w = fma(mreg[q], xb[16 * g + q], w);
            part3[g * M + c] = w;
            __syncthreads();
            xv -= ((part3[c] + part3[M + c]) + part3[2 * M + c]) + part3[3 * M + c];
        }
        if (threadIdx.x < M) {
            put_y(d.xg + (int64_t)k * kYG, c, xv, epoch);
            const int64_t e = (int64_t)perm[k] * kDM + c;
            if (e < P.nF) P.yF[e] = xv;
        }
        // the last back-substitution task to finish gives the verdict: every
        // task's and chain's failure word is ordered before it (the flags'
        // acquires, then this ticket's release sequence) -- and clears the
        // words for the next solve (no pack pass clears them)
        if (threadIdx.x == 0) {
            unsigned* ticket = reinterpret_cast<unsigned*>(d.fail + 4);
            if (__hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nt - 1) {
                P.scal[kScSolveFail] = solve_verdict(d.fail);
                st_wt(d.fail, 0.0);
                st_wt(d.fail + 1, 0.0);
                __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (d.stamps)
                    atomicAdd(d.stamps + 25, __builtin_amdgcn_s_memrealtime() -
                                                 __hip_atomic_load(d.stamps + 26, __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT));
            }
        }
    };
    // Workers take the next task of the order from a shared counter as they
    // finish one (round 6; a fixed round-robin assignment left a worker whose
    // task waited blocking the later tasks assigned to it while others idled).
    // Each worker holds one task at a time and the tasks are taken in order,
    // so the earliest unfinished task is always held by a worker with nothing
    // earlier unfinished: it can run.  The counter grows monotonically over
    // the plan's solves, by ntask + workers per solve (every worker's last
    // take fails once), so solve `epoch` (1, 2, ...) starts at a known base.
    // (Drawing the next ticket when a task starts, to hide the counter's
    // round trip, measured slower: the drawn task then waits for its busy
    // worker while idle ones pass it by -- profiles/r06/f_flow_max.)
    unsigned long long* take = reinterpret_cast<unsigned long long*>(d.fail + 6);
    const unsigned long long base = (unsigned long long)(epoch - 1) * (unsigned long long)(d.ntask + gridDim.x - d.nch);
    int* tsh = sh + 1;
    for (;;) {
        __syncthreads();   // the previous task is done with the LDS tiles (and with tsh)
        if (threadIdx.x == 0)
            *tsh = (int)(__hip_atomic_fetch_add(take, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - base);
        __syncthreads();
        const int t = *tsh;
        if (t >= d.ntask) break;
        task(t);
    }
}

}  // namespace

void dense_setup(DenseArgs& d, const DevProblem& P) {
    d.nt = (int)((P.nF + kDM - 1) / kDM);
    d.np = (int64_t)d.nt * kDM;
}

// ---- the dataflow solve's schedule (round 6) ----------------------------------
// Tile pattern.  Camera blocks b, c (6 rows each, in the plan's order) couple
// only within the half-bandwidth D; the intrinsics rows [nb, nF) couple with
// everything; padding rows (>= nF) with nothing.  So 64-row tiles couple
// within a tile bandwidth w, except the arrow tiles (those holding intrinsics
// rows), which couple with all.
// Order (one level of nested dissection, "twisted"): when the camera tiles
// [0, tc) split as P1 = [0, h), a separator S = [h, h + w) and P2 = [h + w, tc),
// P1 and P2 do not couple.  They are factored at the same time by two chain
// workgroups -- P1 forward, P2 backward (from its far end towards S, so that
// its fill stays in its band and S's rows fill only in P2's last w columns)
// -- and S and the arrow tiles after both, by chain 0.  Permuted order:
// P1, P2 reversed, S, arrow.  The chains are about half as long (the C5
// loop's orbit: nt 29 -> 16 columns on the longer chain).
// Pattern of L: the permuted pattern of S plus its symbolic fill (tile level).
// Chain k links to its previous column p (forms L_kp = A~_kp X_p' itself with
// X_p still in LDS) when L_kp is nonzero and no column j between them needs
// L_kp first (L_kj with L_jp nonzero: T(k, j) would wait for the chain).
// Tasks: D(k) A~_kk, S(k) A~_kp (the chain's inputs, left-looking sums over
// the nonzero L_km, L_pm), T(i, j) L_ij, Y(j) forward, B(k) back substitution.
// Their order: by the earliest start a list schedule with unbounded workers
// gives them (each node's start exceeds its inputs'), so every task waits only
// on earlier tasks and on chain steps that wait only on earlier tasks -- the
// lowest unfinished node can always run (each worker takes tasks in order).

std::vector<char> dense_tile_pattern(const std::vector<ReduceTarget>& targets, int64_t nF, int nt) {
    std::vector<char> e((size_t)nt * nt, 0);
    for (int t = 0; t < nt; ++t) e[(size_t)t * nt + t] = 1;
    for (const ReduceTarget& T : targets) {
        if (T.dst_kind != kDstDense || T.cols < 1) continue;
        const int64_t ld = T.ld > 0 ? T.ld : nF, r0 = T.dst / ld, c0 = T.dst % ld;
        for (int64_t a = r0 / kDM; a <= (r0 + T.rows - 1) / kDM; ++a)
            for (int64_t b = c0 / kDM; b <= (c0 + T.cols - 1) / kDM; ++b)
                e[(size_t)std::max(a, b) * nt + std::min(a, b)] = 1;
    }
    return e;
}

std::vector<int32_t> dense_flow_plan(DenseArgs& d, const DevProblem& P, const std::vector<char>* exact) {
    d.flow = !d.chain && d.nt <= kDenseFlowMaxNt;
    d.nch = d.ntask = 0;
    d.meta_words = 0;
    if (!d.flow) return {};
    const int nt = d.nt;
    // natural tile pattern
    auto cam_range = [&](int t, int& b0, int& b1) {
        const int64_t r0 = (int64_t)t * kDM, r1 = std::min<int64_t>(r0 + kDM, P.nb);
        if (r0 >= r1) return false;
        b0 = (int)(r0 / 6);
        b1 = (int)((r1 - 1) / 6);
        return true;
    };
    auto arrow = [&](int t) { return (int64_t)t * kDM < P.nF && (int64_t)t * kDM + kDM > P.nb; };
    auto couple = [&](int a, int b) {   // natural tiles a > b
        int a0, a1, b0, b1;
        const bool ca = cam_range(a, a0, a1), cb = cam_range(b, b0, b1);
        if (arrow(a) && (cb || arrow(b))) return true;
        if (arrow(b) && ca) return true;
        return ca && cb && a0 - b1 <= P.D;
    };
    int tc = nt, w = 0;
    for (int t = 0; t < nt; ++t)
        if (arrow(t)) { tc = t; break; }
    // Banded arrow (round 6): when the arrow is several tiles and none of them
    // couples with half of the tiles or more (one intrinsics block per
    // camera: reconstruction()'s grouping), the exact tile pattern is banded
    // in a better order than cameras-then-intrinsics -- Cuthill-McKee over the
    // tile graph puts each intrinsics tile among its cameras' tiles -- and
    // nested dissection then splits the whole system into two chains instead
    // of leaving the arrow to chain 0 (RADIAL3 per camera: 30 + 8 columns).
    // ord[k]: the natural tile at banded position k.
    std::vector<int> ord(nt);
    for (int t = 0; t < nt; ++t) ord[t] = t;
    bool banded_arrow = false;
    if (exact && nt - tc >= 3) {
        auto E = [&](int a, int b) { return (*exact)[(size_t)std::max(a, b) * nt + std::min(a, b)] != 0; };
        std::vector<int> deg(nt, 0);
        for (int a = 0; a < nt; ++a)
            for (int b = 0; b < nt; ++b)
                if (a != b && E(a, b)) ++deg[a];
        bool hub = false;
        for (int t = tc; t < nt; ++t) hub = hub || 2 * deg[t] > nt;
        if (!hub) {
            // Cuthill-McKee from tile 0 (an end of the camera band), neighbours
            // by ascending degree, then natural index
            std::vector<int> cm;
            std::vector<char> seen(nt, 0);
            for (int s0 = 0; s0 < nt; ++s0) {
                if (seen[s0]) continue;
                seen[s0] = 1;
                cm.push_back(s0);
                for (size_t q = cm.size() - 1; q < cm.size(); ++q) {
                    std::vector<int> nb;
                    for (int b = 0; b < nt; ++b)
                        if (!seen[b] && E(cm[q], b)) nb.push_back(b);
                    std::stable_sort(nb.begin(), nb.end(), [&](int x, int y) { return deg[x] < deg[y]; });
                    for (int b : nb) {
                        seen[b] = 1;
                        cm.push_back(b);
                    }
                }
            }
            std::vector<int> pos(nt);
            for (int k = 0; k < nt; ++k) pos[cm[k]] = k;
            int wb = 0;
            for (int a = 0; a < nt; ++a)
                for (int b = 0; b < a; ++b)
                    if (E(a, b)) wb = std::max(wb, std::abs(pos[a] - pos[b]));
            if (wb >= 1 && nt - wb - (nt - wb + 1) / 2 >= 2) {
                banded_arrow = true;
                ord = cm;
                tc = nt;
                w = wb;
            }
        }
    }
    if (!banded_arrow)
        for (int a = 0; a < tc; ++a)
            for (int b = 0; b < a; ++b)
                if (couple(a, b)) w = std::max(w, a - b);
    std::vector<int> perm(nt), c0, c1;
    for (int t = 0; t < nt; ++t) perm[t] = ord[t];
    const int len = tc - w, h = (len + 1) / 2, n2 = len - h;
    const bool split = w >= 1 && n2 >= 2;
    if (split) {
        int q = 0;
        for (int t = 0; t < h; ++t) perm[q++] = ord[t];
        for (int t = tc - 1; t >= h + w; --t) perm[q++] = ord[t];
        for (int t = h; t < h + w; ++t) perm[q++] = ord[t];
        for (int t = tc; t < nt; ++t) perm[q++] = ord[t];
        for (int k = 0; k < h; ++k) c0.push_back(k);
        for (int k = h; k < h + n2; ++k) c1.push_back(k);
        for (int k = h + n2; k < nt; ++k) c0.push_back(k);
    } else {
        for (int k = 0; k < nt; ++k) c0.push_back(k);
    }
    // pattern of L (permuted, lower, with fill)
    std::vector<char> nz((size_t)nt * nt, 0);
    auto NZ = [&](int i, int j) -> char& { return nz[(size_t)i * nt + j]; };
    for (int i = 0; i < nt; ++i) {
        NZ(i, i) = 1;
        for (int j = 0; j < i; ++j) {
            const int a = std::max(perm[i], perm[j]), b = std::min(perm[i], perm[j]);
            NZ(i, j) = banded_arrow ? (*exact)[(size_t)a * nt + b] : couple(a, b);
        }
    }
    for (int k = 0; k < nt; ++k)
        for (int i = k + 1; i < nt; ++i)
            if (NZ(i, k))
                for (int j = k + 1; j < i; ++j)
                    if (NZ(j, k)) NZ(i, j) = 1;
    // chains: previous column, link, chain inputs
    std::vector<int> prev(nt, -1), next(nt, -1), info(nt, 0), la(nt, -1);
    for (const auto* c : {&c0, &c1})
        for (size_t q = 1; q < c->size(); ++q) {
            prev[(*c)[q]] = (*c)[q - 1];
            next[(*c)[q - 1]] = (*c)[q];
        }
    auto linked = [&](int k) { return (info[k] & 1) != 0; };
    for (int k = 0; k < nt; ++k) {
        const int p = prev[k];
        bool ln = p >= 0 && NZ(k, p);
        for (int j = p + 1; ln && j < k; ++j)
            if (NZ(j, p) && NZ(k, j)) ln = false;
        if (ln) info[k] |= 1;
        for (int m = 0; m < k; ++m)
            if (NZ(k, m) && !(ln && m == p)) info[k] |= 2;   // D(k) has terms
        for (int m = 0; ln && m < p; ++m)
            if (NZ(k, m) && NZ(p, m)) info[k] |= 4;           // S(k) has terms
        for (int i = k + 1; i < nt && la[k] < 0; ++i)
            if (NZ(i, k)) la[k] = i;
    }
    // tasks and their inputs (node ids: chain step k = k, task t = nt + t)
    std::vector<int32_t> code;
    std::vector<std::vector<int>> dep;
    std::vector<double> dur;
    std::vector<int> t_of((size_t)nt * nt, -1), d_of(nt, -1), s_of(nt, -1), y_of(nt, -1), b_of(nt, -1);
    auto L_node = [&](int i, int j) { return (linked(i) && prev[i] == j) ? i : nt + t_of[(size_t)i * nt + j]; };
    auto X_node = [&](int j) { return (next[j] >= 0 && linked(next[j])) ? next[j] : j; };
    auto add = [&](int kind, int i, int j) {
        code.push_back((kind << 24) | (i << 12) | j);
        dep.emplace_back();
        dur.push_back(1.0);
        return (int)code.size() - 1;
    };
    // create every task first (the inputs refer to them by id)
    for (int k = 0; k < nt; ++k) {
        if (info[k] & 2) d_of[k] = add(kTaskD, k, k);
        if (info[k] & 4) s_of[k] = add(kTaskS, k, prev[k]);
    }
    for (int j = 0; j < nt; ++j)
        for (int i = j + 1; i < nt; ++i)
            if (NZ(i, j) && !(linked(i) && prev[i] == j)) t_of[(size_t)i * nt + j] = add(kTaskT, i, j);
    for (int j = 0; j < nt; ++j) y_of[j] = add(kTaskY, j, j);
    for (int k = 0; k < nt; ++k) b_of[k] = add(kTaskB, k, k);
    // T tasks with no terms (L_ij = A_ij X_j'): a D / S task forms such an
    // L_im itself (pattern bit 1)
    auto t_terms = [&](int i, int j) {
        int n = 0;
        for (int m = 0; m < j; ++m) n += NZ(i, m) && NZ(j, m);
        return n;
    };
    std::vector<char> simple((size_t)nt * nt, 0);
    for (int j = 0; j < nt; ++j)
        for (int i = j + 1; i < nt; ++i)
            if (t_of[(size_t)i * nt + j] >= 0 && t_terms(i, j) == 0) simple[(size_t)i * nt + j] = 1;
    for (size_t t = 0; t < code.size(); ++t) {
        const int kind = code[t] >> 24, i = (code[t] >> 12) & 0xfff, j = code[t] & 0xfff;
        auto& dp = dep[t];
        double terms = 0;
        if (kind == kTaskD || kind == kTaskS || kind == kTaskT) {
            const int jj = kind == kTaskD ? i : j, mend = kind == kTaskD ? i : jj;
            for (int m = 0; m < mend; ++m) {
                if (kind == kTaskD && linked(i) && m == prev[i]) continue;
                if (!NZ(i, m) || !NZ(jj, m)) continue;
                if (kind != kTaskT && simple[(size_t)i * nt + m]) {
                    dp.push_back(X_node(m));
                    if (jj != i) dp.push_back(L_node(jj, m));
                    terms += 2;
                    continue;
                }
                dp.push_back(L_node(i, m));
                if (jj != i) dp.push_back(L_node(jj, m));
                terms += 1;
            }
            if (kind == kTaskT) dp.push_back(X_node(j));
            dur[t] = 2.0 + terms;
        } else if (kind == kTaskY) {
            dp.push_back(X_node(j));
            for (int m = 0; m < j; ++m)
                if (NZ(j, m)) { dp.push_back(L_node(j, m)); dp.push_back(nt + y_of[m]); terms += 1; }
            dur[t] = 1.0 + 0.3 * terms;
        } else {
            dp.push_back(X_node(i));
            dp.push_back(nt + y_of[i]);
            for (int r = i + 1; r < nt; ++r)
                if (NZ(r, i)) { dp.push_back(L_node(r, i)); dp.push_back(nt + b_of[r]); terms += 1; }
            dur[t] = 1.0 + 0.3 * terms;
        }
    }
    // earliest starts (memoised over the DAG; chain steps take 20 units)
    const int nn = nt + (int)code.size();
    std::vector<double> est(nn, -1.0);
    std::vector<char> busy(nn, 0);
    std::function<double(int)> fin = [&](int v) -> double {
        if (est[v] < 0) {
            SFM_REQUIRE(!busy[v], SFM_ERR_UNSUPPORTED, "dense dataflow schedule: cyclic inputs");
            busy[v] = 1;
            double e = 0.0;
            if (v < nt) {
                if (prev[v] >= 0) e = std::max(e, fin(prev[v]));
                if (d_of[v] >= 0) e = std::max(e, fin(nt + d_of[v]));
                if (s_of[v] >= 0) e = std::max(e, fin(nt + s_of[v]));
            } else {
                for (int u : dep[v - nt]) e = std::max(e, fin(u));
            }
            est[v] = e;
        }
        return est[v] + (v < nt ? 20.0 : dur[v - nt]);
    };
    for (int v = 0; v < nn; ++v) fin(v);
    std::vector<int> order(code.size());
    for (size_t t = 0; t < order.size(); ++t) order[t] = (int)t;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        if (est[nt + a] != est[nt + b]) return est[nt + a] < est[nt + b];
        return (code[a] >> 24) < (code[b] >> 24);
    });
    // meta: perm | prev | info | la | chain 0 | chain 1 | lengths (2) | tasks | pattern bytes
    d.nch = c1.empty() ? 1 : 2;
    d.ntask = (int)code.size();
    std::vector<int32_t> meta(6 * (size_t)nt + 2 + code.size() + ((size_t)nt * nt + 3) / 4, 0);
    for (int k = 0; k < nt; ++k) {
        meta[k] = perm[k];
        meta[nt + k] = prev[k];
        meta[2 * nt + k] = info[k];
        meta[3 * nt + k] = la[k];
    }
    for (size_t q = 0; q < c0.size(); ++q) meta[4 * nt + q] = c0[q];
    for (size_t q = 0; q < c1.size(); ++q) meta[5 * nt + q] = c1[q];
    meta[6 * nt] = (int32_t)c0.size();
    meta[6 * nt + 1] = (int32_t)c1.size();
    for (size_t q = 0; q < order.size(); ++q) meta[6 * nt + 2 + q] = code[order[q]];
    for (size_t e = 0; e < nz.size(); ++e) nz[e] = (char)(nz[e] | (simple[e] ? 2 : 0));
    std::memcpy(meta.data() + 6 * nt + 2 + code.size(), nz.data(), nz.size());
    d.meta_words = (int64_t)meta.size();
    return meta;
}

// flags: x (nt), L tiles + chain inputs (2 nt^2), y (nt); then (8-byte
// aligned) the dataflow back substitution's tagged x granules (kYG per column)
static size_t dense_granule_word(const DenseArgs& d) { return ((size_t)d.nt + 2 * (size_t)d.nt * d.nt + d.nt + 1) & ~(size_t)1; }
size_t dense_flag_words(const DenseArgs& d) { return dense_granule_word(d) + 2 * (size_t)kYG * d.nt; }

size_t dense_doubles(const DenseArgs& d) {
    // A | X | b y x | fail (8) | flags and granules | the dataflow schedule
    return (size_t)d.np * d.np + (size_t)d.nt * kDM * kDM + 3 * (size_t)d.np + 8 + (dense_flag_words(d) + 1) / 2 + 2 +
           ((size_t)d.meta_words + 1) / 2 + 1;
}

void dense_bind(DenseArgs& d, double* base) {
    d.A = base;
    d.X = d.A + (size_t)d.np * d.np;
    d.b = d.X + (size_t)d.nt * kDM * kDM;
    d.y = d.b + d.np;
    d.x = d.y + d.np;
    d.fail = d.x + d.np;
    d.xflag = reinterpret_cast<unsigned*>(d.fail + 8);   // zeroed by the caller once
    d.fflag = d.xflag + d.nt;
    d.xg = reinterpret_cast<unsigned long long*>(d.xflag + dense_granule_word(d));
    d.meta = reinterpret_cast<const int32_t*>(d.xflag + ((dense_flag_words(d) + 1) & ~(size_t)1));
}

void dense_solve(const DenseArgs& d, const DevProblem& P, double radius, hipStream_t s, unsigned epoch) {
    const size_t lds_p = (3 * M * LD + 2) * sizeof(double), lds_u = 2 * M * kUpdLD * sizeof(double);
    set_dyn_lds((const void*)dense_panel_kernel, lds_p);
    set_dyn_lds((const void*)dense_update_kernel, lds_u);
    const int n_cu = device_cu_count();
    // up to kDenseFlowMaxNt block columns the dataflow kernel (round 6, with
    // the host schedule and the lookahead back substitution: RADIAL3 per
    // camera 480 -> 540, dense-S 110 -> 112 LM-iters/s against the launch
    // chain, profiles/r06/f_flow_max); the launch chain stays the form for
    // wider systems (and every system under SFM_CTX_BA_DENSE_CHAIN)
    if (d.flow) {
        // factorisation and both substitutions in one dataflow launch: the
        // chain workgroups and up to n_cu - nch task workers, one workgroup
        // per CU (the LDS request forces it): a chain's pivot wave must not
        // share its SIMD with another workgroup's fp64 MFMAs, which stall its
        // fp64 VALU (15x in tools/probe/diag16_probe.hip), and every workgroup
        // is resident, so every wait ends
        const size_t lds_f = std::max<size_t>(kDfLds * sizeof(double), 81 * 1024);
        set_dyn_lds((const void*)dense_flow_kernel, lds_f);
#ifndef SFM_DF_WORKER_DIV
#define SFM_DF_WORKER_DIV 1   // (A/B only: fewer task workers)
#endif
        const int workers = std::min(d.ntask, (n_cu - d.nch) / SFM_DF_WORKER_DIV);
        hipLaunchKernelGGL(dense_flow_kernel, dim3(d.nch + workers), dim3(NT), lds_f, s, d, P, radius, epoch);
        SFM_HIP(hipGetLastError());
        return;
    }
    // block columns in groups of W = kDenseW: panel c, then the group's
    // later columns updated from column c alone (rhs of column c fused), ...;
    // after the group's last panel every later tile is updated from all W
    // columns in one pass, read and written once
    constexpr int W = kDenseW;
    for (int k = 0; k < d.nt; k += W) {
        const int w = std::min(W, d.nt - k);
        for (int c = k; c < k + w; ++c) {
            hipLaunchKernelGGL(dense_panel_kernel, dim3(d.nt - c), dim3(NT), lds_p, s, d, P, radius, c);
            SFM_HIP(hipGetLastError());
            const int m = d.nt - c - 1;   // rows below column c
            if (c + 1 < k + w) {
                const int nw = k + w - c - 1, n_tiles = nw * m;
                hipLaunchKernelGGL(dense_update_kernel, dim3(n_tiles + m), dim3(NT), lds_u, s, d, P, radius, c, 1,
                                   c + 1, n_tiles, nw, c);
                SFM_HIP(hipGetLastError());
            }
        }
        const int m2 = d.nt - k - w;   // trailing block columns
        if (m2 > 0) {
            const int n_tiles = m2 * (m2 + 1) / 2;
            hipLaunchKernelGGL(dense_update_kernel, dim3(n_tiles + m2), dim3(NT), lds_u, s, d, P, radius, k, w, k + w,
                               n_tiles, 0, k + w - 1);
            SFM_HIP(hipGetLastError());
        }
    }
    if (d.nt <= n_cu && !d.chain) {
        // one workgroup per block column, all resident: more than half a CU's
        // LDS each, so one per CU
        constexpr size_t lds_all = (3 * M * LD + 15 * M) * sizeof(double);
        static_assert(lds_all > 80 * 1024 && lds_all <= 160 * 1024, "one back-substitution workgroup per CU");
        set_dyn_lds((const void*)dense_back_all_kernel, lds_all);
        hipLaunchKernelGGL(dense_back_all_kernel, dim3(d.nt), dim3(NT), lds_all, s, d, P, epoch);
        SFM_HIP(hipGetLastError());
        return;
    }
    for (int k = d.nt - 1; k >= 0; --k) {
        hipLaunchKernelGGL(dense_back_kernel, dim3(k > 0 ? k : 1), dim3(NT), 0, s, d, P, k);
        SFM_HIP(hipGetLastError());
    }
}

}  // namespace sfm
