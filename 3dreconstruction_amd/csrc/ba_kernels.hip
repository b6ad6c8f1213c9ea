// Bundle-adjustment kernels for CDNA4 (gfx950), fp64 throughout.
//
// Reference: src/adjuster/BundleAdjuster.h — ReprojectCost :33-69 (pinhole,
// ceres::AngleAxisRotatePoint), HuberLoss(4) :109, ceres::Solve with
// SPARSE_SCHUR (point blocks eliminated) :125-126, 167-174; residual models
// SnavelyReprojectionError.h:16-54 and OpenMVG PINHOLE_CAMERA_RADIAL3
// (sparseBuilder.cpp:1292-1299) through the CM template parameter.
//
// One LM iteration on device:
//   campre      per-camera rotation terms (sin/cos once per camera, not per obs)
//   image_gram  per image (WGs): U = J_F' J_F over its observations (pose 6 |
//               intrinsics 4 or 6), b = J_F' f, cost 1/2 sum rho   [after an
//               accepted step only]
//   schur       chunk points, per chunk (one wave): observations -> corrected,
//               Jacobi-scaled Jacobians (VALU) -> per point V + D^2, Cholesky
//               L, w = L^-1 g -> Z = W L^-T into an LDS panel -> the chunk tile
//               -Z Z' (and -Z w) on the fp64 MFMA (v_mfma_f64_16x16x4_f64),
//               lower 16x16 tiles only
//   zpoint      general points, per point (one wave): the same elimination,
//               Z rows to a global buffer (product terms, preduce_*)
//   reduce      static gather plan: tiles + image blocks (+ products) -> RCS
//   solve       band + arrow: block cyclic reduction (ba_bcr.hip; solve_kernel
//               is the one-workgroup fallback); dense: blocked Cholesky
//   cand/step   candidate cameras; per point back-substitution y_E =
//               L^-T (w - Z' y_F), model cost change, candidate cost
//   finalize    fixed-order reduction of per-block partials (deterministic)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>

#include "ba_cand.h"
#include "ba_kernels.h"
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


typedef double v4d __attribute__((ext_vector_type(4)));

// doubles per intrinsics block of a residual model (RADIAL3: f, ppx, ppy, k1-k3)
template <int CM>
constexpr int kIW = CM == SFM_CAM_RADIAL3 ? 6 : 4;

// 1/sqrt(d): hardware estimate + two Newton steps (full fp64 accuracy)
// 1/d: hardware estimate + two Newton steps
__device__ __forceinline__ double rcp_nr(double d) {
    double y = __builtin_amdgcn_rcp(d);
#pragma unroll
    for (int it = 0; it < 2; ++it) y = fma(y, fma(-d, y, 1.0), y);
    return y;
}

__device__ __forceinline__ double rsqrt_nr(double d) {
    double y = __builtin_amdgcn_rsq(d);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const double hy = 0.5 * d * y;
        y = fma(y, fma(-hy, y, 0.5), y);
    }
    return y;
}

__device__ __forceinline__ double clampd(double v, double lo, double hi) {
    return fmin(fmax(v, lo), hi);
}

// LM damping of a point-block diagonal entry: D^2 = clamp(diag) / radius.
// Ceres forms D = sqrt(clamp(diag) / radius) and adds D * D (the oracle does
// the same); the square of the rounded square root differs from its argument
// by about an ulp, and dropping the sqrt takes three dependent sqrt sequences
// off the point factorisation's critical path (Schur 0.347 -> 0.335 ms at
// C4).  Every point kernel (Schur, step, general points) uses this formula,
// so the elimination and the back substitution see the same V + D^2.  The
// camera columns keep Ceres's form (formed once per RCS, not per point).
__device__ __forceinline__ double point_d2(const DevProblem& P, double diag, double inv_radius) {
    return clampd(diag, P.min_diag, P.max_diag) * inv_radius;
}

// ---------------------------------------------------------------------------
// per-camera precompute (make_campre: ba_cand.h)
// ---------------------------------------------------------------------------
__global__ void campre_kernel(const double* __restrict__ extr, int n, CamPre* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double e[6];
    for (int a = 0; a < 6; ++a) e[a] = extr[6 * (size_t)i + a];
    out[i] = make_campre(e);
}

// ---------------------------------------------------------------------------
// residual + loss-corrected Jacobian of one observation
// (BundleAdjuster.h:40-65 model; ceres Corrector with rho'' <= 0: r and J
// scaled by sqrt(rho'))
// ---------------------------------------------------------------------------
template <int IW>
struct LinW {
    double f[2];
    double Jc[2][6];
    double Ji[2][IW];
    double Jx[2][3];
    double half_rho;
    bool ok;
};
using Lin = LinW<4>;
template <int CM>
using LinT = LinW<kIW<CM>>;

template <int CM, bool JC, bool JI, bool JX>
__device__ __forceinline__ void linearize(const CamPre& cp, const double* in, const double* X, double u0,
                                          double u1, double huber_a, LinT<CM>& L) {
    double P[3];
    const double* u = cp.u;
    const double cr0 = u[1] * X[2] - u[2] * X[1], cr1 = u[2] * X[0] - u[0] * X[2],
                 cr2 = u[0] * X[1] - u[1] * X[0];
    if (cp.small != 0.0) {
        P[0] = X[0] + cr0; P[1] = X[1] + cr1; P[2] = X[2] + cr2;
    } else {
        const double tmp = (u[0] * X[0] + u[1] * X[1] + u[2] * X[2]) * cp.omc;
        P[0] = X[0] * cp.c + cr0 * cp.s + u[0] * tmp;
        P[1] = X[1] * cp.c + cr1 * cp.s + u[1] * tmp;
        P[2] = X[2] * cp.c + cr2 * cp.s + u[2] * tmp;
    }
    P[0] += cp.t[0]; P[1] += cp.t[1]; P[2] += cp.t[2];
    // one reciprocal for the projection and its Jacobian (x = P0/P2 to about
    // 1 ulp): v_rcp + two Newton steps, a shorter dependent chain than the
    // IEEE division sequence (C4 +0.6 % LM iterations/s)
    const double iz = rcp_nr(P[2]);
    double r0, r1;
    // unscaled dr/dP (2x3) and dr/d(intrinsics) (2 x kIW) of the model
    double A[2][3], Ji[2][kIW<CM>];
    if constexpr (CM == SFM_CAM_RADIAL3) {
        // OpenMVG ResidualErrorFunctor_Pinhole_Intrinsic_Radial_K3: (x, y) = P/P2,
        // c = 1 + k1 r2 + k2 r2^2 + k3 r2^3, r = pp + f c (x, y) - obs;
        // dr/dP = f [c I + D (x, y)(x, y)'] dp/dP with D = 2 (k1 + 2 k2 r2 + 3 k3 r2^2),
        // dp/dP = 1/P2 [1 0 -x; 0 1 -y]
        const double xu = P[0] * iz, yu = P[1] * iz;
        const double r2 = xu * xu + yu * yu, r4 = r2 * r2, r6 = r4 * r2;
        const double rc = 1.0 + in[3] * r2 + in[4] * r4 + in[5] * r6;
        r0 = in[1] + in[0] * (xu * rc) - u0;
        r1 = in[2] + in[0] * (yu * rc) - u1;
        if (JC || JI || JX) {
            const double dd = 2.0 * (in[3] + 2.0 * in[4] * r2 + 3.0 * in[5] * r4);
            const double b01 = in[0] * dd * xu * yu;
            const double B[2][2] = {{in[0] * (rc + dd * xu * xu), b01}, {b01, in[0] * (rc + dd * yu * yu)}};
            const double pu[2] = {xu, yu};
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                A[r][0] = iz * B[r][0];
                A[r][1] = iz * B[r][1];
                A[r][2] = -iz * (B[r][0] * xu + B[r][1] * yu);
                Ji[r][0] = pu[r] * rc;
                Ji[r][1] = r == 0 ? 1.0 : 0.0;
                Ji[r][2] = r == 1 ? 1.0 : 0.0;
                Ji[r][3] = in[0] * pu[r] * r2;
                Ji[r][4] = in[0] * pu[r] * r4;
                Ji[r][5] = in[0] * pu[r] * r6;
            }
        }
    } else if constexpr (CM == SFM_CAM_SNAVELY) {
        // SnavelyReprojectionError.h:31-47: p = -P/P2, d = 1 + r2 (l1 + l2 r2),
        // r = f d p - obs; dr/dP = f [d I + 2 (l1 + 2 l2 r2) p p'] dp/dP with
        // dp/dP = -1/P2 [1 0 xp; 0 1 yp]
        const double xp = -P[0] * iz, yp = -P[1] * iz;
        const double r2 = xp * xp + yp * yp;
        const double d = 1.0 + r2 * (in[1] + in[2] * r2);
        r0 = in[0] * d * xp - u0;
        r1 = in[0] * d * yp - u1;
        if (JC || JI || JX) {
            const double dd2 = 2.0 * (in[1] + 2.0 * in[2] * r2);
            const double b01 = in[0] * dd2 * xp * yp;
            const double B[2][2] = {{in[0] * (d + dd2 * xp * xp), b01}, {b01, in[0] * (d + dd2 * yp * yp)}};
            const double pp[2] = {xp, yp};
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                A[r][0] = -iz * B[r][0];
                A[r][1] = -iz * B[r][1];
                A[r][2] = -iz * (B[r][0] * xp + B[r][1] * yp);
                Ji[r][0] = d * pp[r];
                Ji[r][1] = in[0] * r2 * pp[r];
                Ji[r][2] = in[0] * r2 * r2 * pp[r];
                Ji[r][3] = 0.0;
            }
        }
    } else {
        const double x = P[0] * iz, y = P[1] * iz;
        r0 = in[0] * x + in[2] - u0;
        r1 = in[1] * y + in[3] - u1;
        A[0][0] = in[0] * iz; A[0][1] = 0.0; A[0][2] = -in[0] * x * iz;
        A[1][0] = 0.0; A[1][1] = in[1] * iz; A[1][2] = -in[1] * y * iz;
        Ji[0][0] = x; Ji[0][1] = 0.0; Ji[0][2] = 1.0; Ji[0][3] = 0.0;
        Ji[1][0] = 0.0; Ji[1][1] = y; Ji[1][2] = 0.0; Ji[1][3] = 1.0;
    }
    L.ok = isfinite(r0) && isfinite(r1);
    const double sq = r0 * r0 + r1 * r1;
    double rho0, sr = 1.0;   // Huber: rho' = 1 (inlier) needs no square root
    if (huber_a > 0.0 && sq > huber_a * huber_a) {
        const double rr = sqrt(sq);
        rho0 = 2.0 * huber_a * rr - huber_a * huber_a;
        sr = sqrt(fmax(DBL_MIN, huber_a / rr));
    } else {
        rho0 = sq;
    }
    L.half_rho = 0.5 * rho0;
    L.f[0] = r0 * sr; L.f[1] = r1 * sr;
    if (JC || JI || JX) {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int k = 0; k < 3; ++k) A[r][k] *= sr;
        if (JI) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int k = 0; k < kIW<CM>; ++k) L.Ji[r][k] = Ji[r][k] * sr;
        }
        // dP/dX = R; dP/dw = -Al [X]x Ar with Al = R (Rodrigues) or I (small
        // angle), so the left factor A Al is J_X itself or A.
        double Jx[2][3];
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                Jx[r][j] = A[r][0] * cp.R[j] + A[r][1] * cp.R[3 + j] + A[r][2] * cp.R[6 + j];
        if (JX) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int j = 0; j < 3; ++j) L.Jx[r][j] = Jx[r][j];
        }
        if (JC) {
            double N[9];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                N[0 + j] = -X[2] * cp.Ar[3 + j] + X[1] * cp.Ar[6 + j];
                N[3 + j] = X[2] * cp.Ar[0 + j] - X[0] * cp.Ar[6 + j];
                N[6 + j] = -X[1] * cp.Ar[0 + j] + X[0] * cp.Ar[3 + j];
            }
            const bool small = cp.small != 0.0;
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                double B[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) B[k] = small ? A[r][k] : Jx[r][k];
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    L.Jc[r][j] = -(B[0] * N[j] + B[1] * N[3 + j] + B[2] * N[6 + j]);
                    L.Jc[r][3 + j] = A[r][j];
                }
            }
        }
    }
}

// Global-address-space agent-scope accesses for values handed between
// workgroups of one launch (sc1: written through / read past this CU's L1;
// cdna_hip_programming.md Guideline 16, counter form)
typedef __attribute__((address_space(1))) unsigned gu32_t;
typedef __attribute__((address_space(1))) double gf64_t;
__device__ __forceinline__ void st_wt64(double* p, double v) {
    __hip_atomic_store((gf64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt64(const double* p) {
    return __hip_atomic_load((gf64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// block reduction helpers (256 threads, fixed order => deterministic)
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void wave_sum(double (&v)[N]) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] += __shfl_xor(v[k], o);
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}

// ---------------------------------------------------------------------------
// per-image Gram blocks: U = J_F' J_F (10x10), b = J_F' f, cost
// P.gram_seg (<= kGramSeg) workgroups per image, one observation per lane per step.  Each lane
// keeps its own running sums of the 62 structurally nonzero entries of
// [J_c | J_i | f]' [J_c | J_i | f] (J_i row 0 = [x s, 0, s, 0], row 1 =
// [0, y s, 0, s]) plus the cost on the VALU -- 90 FMAs per observation, no
// LDS staging -- and the wave then reduce-scatters the 64 sums (permlane32 /
// permlane16 swaps, then xor shuffles) so lane l ends with entry l; the four
// waves add in fixed order.
// ---------------------------------------------------------------------------
namespace gram {
// F columns of an image block: pose 6 | intrinsics kIW; index FW is f
template <int CM>
constexpr int FW = 6 + kIW<CM>;
// structurally nonzero entries of [J_c | J_i | f] rows 0 / 1 (index 0..FW)
// PINHOLE: J_i row 0 = [x s, 0, s, 0], row 1 = [0, y s, 0, s];
// SNAVELY: J_i rows = [d, f r2, f r2^2, 0] p_r s (column 9 is never a parameter);
// RADIAL3: J_i row 0 = [x c, 1, 0, f x r2, f x r4, f x r6] s, row 1 the same
//          with y and (0, 1) at the principal point
template <int CM>
constexpr bool in0(int i) {
    return CM == SFM_CAM_RADIAL3 ? i != 8 : CM == SFM_CAM_SNAVELY ? i != 9 : (i < 6 || i == 6 || i == 8 || i == 10);
}
template <int CM>
constexpr bool in1(int i) {
    return CM == SFM_CAM_RADIAL3 ? i != 7 : CM == SFM_CAM_SNAVELY ? i != 9 : (i < 6 || i == 7 || i == 9 || i == 10);
}
struct Slots {
    int i[128], j[128], id[13][13], n;
};
template <int CM>
constexpr Slots make_slots() {
    Slots t{};
    t.n = 0;
    for (int a = 0; a < 13; ++a)
        for (int b = 0; b < 13; ++b) t.id[a][b] = -1;
    for (int a = 0; a <= FW<CM>; ++a)
        for (int b = 0; b <= a; ++b)
            if ((in0<CM>(a) && in0<CM>(b)) || (in1<CM>(a) && in1<CM>(b))) {
                t.i[t.n] = a; t.j[t.n] = b;
                t.id[a][b] = t.id[b][a] = t.n;
                ++t.n;
            }
    return t;
}
template <int CM>
struct SlotTable {
    static constexpr Slots kS = make_slots<CM>();
    static constexpr int kCost = kS.n;   // slot of the cost; later slots stay zero
    static constexpr int kPasses = (kS.n + 1 + 63) / 64;   // 64 register sums per lane and pass
};
static_assert(SlotTable<SFM_CAM_PINHOLE>::kS.n == 62, "image Gram: 62 nonzero entries (pinhole)");
static_assert(SlotTable<SFM_CAM_SNAVELY>::kS.n == 55, "image Gram: 55 nonzero entries (Snavely)");
static_assert(SlotTable<SFM_CAM_RADIAL3>::kS.n == 90 && SlotTable<SFM_CAM_RADIAL3>::kPasses == 2,
              "image Gram: 90 nonzero entries in two passes (RADIAL3)");

__device__ __forceinline__ unsigned lo32(double v) { return (unsigned)__double_as_longlong(v); }
__device__ __forceinline__ unsigned hi32(double v) { return (unsigned)(__double_as_longlong(v) >> 32); }
__device__ __forceinline__ double mk(unsigned lo, unsigned hi) {
    return __longlong_as_double(((long long)hi << 32) | lo);
}
// v[j] + partner's v[j] in the lanes that keep j, v[j+H] + partner's in the others
template <int H>
__device__ __forceinline__ void swap_add(double (&v)[64]) {
#pragma unroll
    for (int k = 0; k < H; ++k) {
        const double a = v[k], b = v[k + H];
        double na, nb;
        if (H == 32) {
            const auto l = __builtin_amdgcn_permlane32_swap(lo32(a), lo32(b), false, false);
            const auto h = __builtin_amdgcn_permlane32_swap(hi32(a), hi32(b), false, false);
            na = mk(l[0], h[0]); nb = mk(l[1], h[1]);
        } else {
            const auto l = __builtin_amdgcn_permlane16_swap(lo32(a), lo32(b), false, false);
            const auto h = __builtin_amdgcn_permlane16_swap(hi32(a), hi32(b), false, false);
            na = mk(l[0], h[0]); nb = mk(l[1], h[1]);
        }
        v[k] = na + nb;
    }
}
template <int M>
__device__ __forceinline__ void xor_add(double (&v)[64], int lane) {
    const bool up = (lane & M) != 0;
#pragma unroll
    for (int k = 0; k < M; ++k) {
        const double send = up ? v[k] : v[k + M], keep = up ? v[k + M] : v[k];
        v[k] = keep + __shfl_xor(send, M);
    }
}
// after the call lane l holds the wave sum of v[l] in v[0]
__device__ __forceinline__ void reduce_scatter64(double (&v)[64], int lane) {
    swap_add<32>(v);   // lanes 0-31: entries 0..31, lanes 32-63: 32..63 (in v[0..31])
    swap_add<16>(v);   // row r (16 lanes): entries 16 r + (0..15)
    xor_add<8>(v, lane);
    xor_add<4>(v, lane);
    xor_add<2>(v, lane);
    xor_add<1>(v, lane);
}
}  // namespace gram

// PASS: which 64 slots this launch sums (RADIAL3's 91 sums take two passes,
// each re-linearising the image's observations; the other models one).
template <int CM, int PASS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void image_gram_kernel(DevProblem P, const CamPre* __restrict__ cps,
                                                         const double* __restrict__ intr,
                                                         const double* __restrict__ X,
                                                         const double* __restrict__ gate) {
    if (gate && *gate == 0.0) return;   // speculative pass, step not accepted (uniform)
    using kT = gram::SlotTable<CM>;
    constexpr int IW = kIW<CM>, FW = gram::FW<CM>, S0 = 64 * PASS;
    constexpr bool kHasCost = kT::kCost >= S0 && kT::kCost < S0 + 64;
    // workgroup -> (image with observations, slice); outputs at b = img * ns + seg
    const int ns = P.gram_seg, gi = blockIdx.x / ns, seg = blockIdx.x - ns * gi, img = P.gram_img[gi];
    const int b = img * ns + seg;
    const int a0 = P.img_obs_ptr[img], n = P.img_obs_ptr[img + 1] - a0;
    const int o0 = a0 + (int)((int64_t)n * seg / ns), o1 = a0 + (int)((int64_t)n * (seg + 1) / ns);
    const int colc = P.img_colc[img], coli = P.img_coli[img];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __shared__ CamPre scp;
    __shared__ double sin_[IW], ssc[FW];
    __shared__ double part[4][64], badw[4];
    if (threadIdx.x < sizeof(CamPre) / 8)
        reinterpret_cast<double*>(&scp)[threadIdx.x] = reinterpret_cast<const double*>(&cps[img])[threadIdx.x];
    if (threadIdx.x >= 64 && threadIdx.x < 64 + IW)
        sin_[threadIdx.x - 64] = intr[IW * (size_t)P.img_intr[img] + threadIdx.x - 64];
    if (threadIdx.x >= 96 && threadIdx.x < 96 + FW) {
        const int a = threadIdx.x - 96;
        ssc[a] = a < 6 ? (colc >= 0 ? P.scaleF[colc + a] : 0.0) : P.scaleF[coli + a - 6];
    }
    __syncthreads();
    double g[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) g[k] = 0.0;
    double bad = 0.0;
    // software pipeline: point ids / measurements two iterations ahead, the
    // point itself one iteration ahead
    auto fetch_ids = [&](int base, int& p, double2& uv) {
        const int q = base + lane;
        p = q < o1 ? P.img_pt[q] : -1;
        uv = q < o1 ? reinterpret_cast<const double2*>(P.img_uv)[q] : double2{0.0, 0.0};
    };
    auto fetch_x = [&](int p, double (&x)[3]) {
#pragma unroll
        for (int a = 0; a < 3; ++a) x[a] = p >= 0 ? X[3 * (size_t)p + a] : 0.0;
    };
    // one observation's contribution (lane's running sums, observation order)
    auto process = [&](int p_cur, const double2& uv, const double (&Xp)[3]) {
    // re-read the staged camera from LDS each step instead of keeping its
    // 28 doubles live across the loop (register budget of 2 waves/SIMD)
    asm volatile("" ::: "memory");
    if (p_cur >= 0) {
        LinT<CM> L;
        linearize<CM, true, true, false>(scp, sin_, Xp, uv.x, uv.y, P.huber_a, L);
        if constexpr (kHasCost) g[kT::kCost - S0] += L.half_rho;
        bad = fmax(bad, L.ok ? 0.0 : 1.0);
        // unscaled rows; the per-image column scales are applied to the sums
        auto r = [&](int q, int i) -> double {
            return i < 6 ? L.Jc[q][i] : i < FW ? L.Ji[q][i - 6] : L.f[q];
        };
#pragma unroll
        for (int s = 0; s < 64; ++s) {
            if (S0 + s >= kT::kS.n) break;
            const int i = kT::kS.i[S0 + s], j = kT::kS.j[S0 + s];
            if (gram::in0<CM>(i) && gram::in0<CM>(j)) g[s] = fma(r(0, i), r(0, j), g[s]);
            if (gram::in1<CM>(i) && gram::in1<CM>(j)) g[s] = fma(r(1, i), r(1, j), g[s]);
        }
    }
    };
    // three stages: the point gather (random rows of X) two iterations ahead
    int p_c, p_n, p_nn;
    double2 uv_c, uv_n, uv_nn;
    double x_c[3], x_n[3];
    fetch_ids(o0 + 64 * wave, p_c, uv_c);
    fetch_ids(o0 + 64 * wave + 256, p_n, uv_n);
    fetch_ids(o0 + 64 * wave + 512, p_nn, uv_nn);
    fetch_x(p_c, x_c);
    fetch_x(p_n, x_n);
    for (int base = o0 + 64 * wave; base < o1; base += 256) {
        const int p_cur = p_c;
        const double2 uv = uv_c;
        const double Xp[3] = {x_c[0], x_c[1], x_c[2]};
        p_c = p_n; uv_c = uv_n;
        x_c[0] = x_n[0]; x_c[1] = x_n[1]; x_c[2] = x_n[2];
        p_n = p_nn; uv_n = uv_nn;
        fetch_x(p_n, x_n);
        fetch_ids(base + 768, p_nn, uv_nn);
        process(p_cur, uv, Xp);
    }
    gram::reduce_scatter64(g, lane);
    bad = wave_max(bad);
    part[wave][lane] = g[0];
    if (lane == 0) badw[wave] = bad;
    __syncthreads();
    // slot s of this pass (S0 <= s < S0 + 64) summed over the four waves
    auto tot = [&](int s) { return ((part[0][s - S0] + part[1][s - S0]) + part[2][s - S0]) + part[3][s - S0]; };
    auto mine = [&](int s) { return s >= S0 && s < S0 + 64; };
    if (threadIdx.x < FW * FW) {
        const int i = threadIdx.x / FW, j = threadIdx.x % FW, s = kT::kS.id[i][j];
        if (s >= 0 ? mine(s) : PASS == 0) {
            const double u = s >= 0 ? ssc[i] * ssc[j] * tot(s) : 0.0;
            P.U[(size_t)b * (FW * FW) + threadIdx.x] = u;
            if (i == j) P.Ucn[(size_t)b * FW + i] = u;
        }
    }
    if (threadIdx.x >= 160 && threadIdx.x < 160 + FW) {
        const int i = threadIdx.x - 160, s = kT::kS.id[FW][i];
        if (mine(s)) P.Ub[(size_t)b * FW + i] = ssc[i] * tot(s);
    }
    if (kHasCost && threadIdx.x == 192) {
        P.part_u[2 * (size_t)b] = tot(kT::kCost);
        P.part_u[2 * (size_t)b + 1] = fmax(fmax(badw[0], badw[1]), fmax(badw[2], badw[3]));
    }
}

// Iteration 0 after the Jacobi scales are known: the image Gram pass applies
// the per-image column scales to its sums (u = (s_i s_j) * sum), so the
// scaled blocks follow from the unit-scale pass's exactly, without a second
// linearisation of every observation (bit-identical to re-running the pass).
template <int CM>
__global__ __launch_bounds__(128) void gram_rescale_kernel(DevProblem P) {
    using kT = gram::SlotTable<CM>;
    constexpr int FW = gram::FW<CM>;
    const int gi = blockIdx.x / P.gram_seg, img = P.gram_img[gi];
    const int b = img * P.gram_seg + (blockIdx.x - gi * P.gram_seg);
    const int colc = P.img_colc[img], coli = P.img_coli[img];
    __shared__ double ssc[FW];
    if (threadIdx.x < FW) {
        const int a = threadIdx.x;
        ssc[a] = a < 6 ? (colc >= 0 ? P.scaleF[colc + a] : 0.0) : P.scaleF[coli + a - 6];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < FW * FW; e += 128) {
        const int i = e / FW, j = e % FW, s = kT::kS.id[i][j];
        const double u = s >= 0 ? ssc[i] * ssc[j] * P.U[(size_t)b * (FW * FW) + e] : 0.0;
        P.U[(size_t)b * (FW * FW) + e] = u;
        if (i == j) P.Ucn[(size_t)b * FW + i] = u;
    }
    if (threadIdx.x < FW) {
        const int i = threadIdx.x;
        P.Ub[(size_t)b * FW + i] = ssc[i] * P.Ub[(size_t)b * FW + i];
    }
}

__global__ void fill_kernel(double* p, int64_t n, double v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

// up to kSegs copies (src) or fills (src null: value v) in one launch, grid-stride
__global__ void segs_kernel(SegList L) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = 0; k < L.n; ++k) {
        const Seg& g = L.seg[k];
        for (int64_t j = i; j < g.n; j += stride) g.dst[j] = g.src ? g.src[j] : g.v;
    }
}

__global__ void fscale_kernel(DevProblem P) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < P.nF) P.scaleF[c] = 1.0 / (1.0 + sqrt(P.cnF[c]));
}

// ---------------------------------------------------------------------------
// Schur chunk kernel: one workgroup per tile group, one wavefront per chunk
//
// A tile group's chunks (<= kGroupChunks) share one slot layout.  Each wave
// owns its chunk's whole 80x80 tile as 15 lower 16x16 fp64 MFMA accumulators
// and walks the chunk in batches of <= kSubPts points / <= kSubObs (= 64)
// observations:
//   A  lane = observation: linearise, Jacobi-scale, stage Jx | f | J_intr
//   B  lane = point: V + D^2, Cholesky, L^-1, w = L^-1 g  (panel row 79)
//   C  lane = observation: M = Jx L^-T, camera rows of Z = J_c' M
//   C2 lane = (point, column): intrinsics rows of Z, ordered sum
//   D  tile -= panel panel' : ceil(3 npts / 4) k-steps x 15 MFMAs
// Inside the batch loop each wave syncs only itself (its LDS is its own), so
// co-resident waves overlap each other's VALU and MFMA phases; at the end the
// group's waves add their tiles in LDS in wave order and wave 0 writes the
// group's one tile.  Every sum has a fixed order, so results are
// bit-reproducible.
// ---------------------------------------------------------------------------

__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// wave-local LDS exchange: every lane's writes visible to the wave
// (LDS-only fences: the exchange is through LDS, so the fences need not
// order, or wait for, the wave's global accesses -- e.g. a prefetch in flight)
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// LDS copy of a CamPre padded to 240 B (60 dwords): lanes of a batch read up
// to 10 different cameras' fields at once, and a 60-dword stride puts their
// 16-byte reads on disjoint banks (224 B = 56 dwords collided: 56 * 8 = 0 mod 64)
struct alignas(16) CamPreL {
    CamPre cp;
    double pad[2];
};
// next wave batch from p0: <= kSubPts points and <= kSubObs observations
// (cpoff = chunk-relative point offsets in LDS); returns its point count
template <int SP = kSubPts, int SO = kSubObs>
__device__ __forceinline__ int batch_points(const int* cpoff, int p0, int np) {
    const int lane = threadIdx.x & 63, q1 = p0 + 1 + lane;
    const bool fits = lane < SP && q1 <= np && cpoff[q1] - cpoff[p0] <= SO;
    return __builtin_ctzll(~__ballot(fits));
}

// staged camera t is optimised (has F columns); constant images are not
__device__ __forceinline__ bool crow_valid(const ChunkDesc& cd, int t) { return cd.cam_col[t] >= 0; }

// lower 16x16 tiles (ti >= tj) of the NT x NT tile grid, row-major
__device__ constexpr int kTi[15] = {0, 1, 1, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 4};
__device__ constexpr int kTj[15] = {0, 0, 1, 0, 1, 2, 0, 1, 2, 3, 0, 1, 2, 3, 4};


// NT = 5: rows 0..75 F blocks, row 79 = w, so -Z w comes out of the MFMA.
// NT = 4: rows 0..63 F blocks; -Z w (64 values) is a VALU dot product per lane.
// SP / SO: points / observations per wave batch.  The panel holds 3 columns
// per point padded to the MFMA k of 4 and NT*16 rows (NT = 4 keeps w apart).
// SE: the solve's first pass also forms the Jacobi point scales (what
// point_scale_kernel computes) from the unscaled Jx it linearises anyway,
// writes them to scaleE and uses them, instead of a separate pass.
template <int CM, int NT, int SP = kSubPts, int SO = kSubObs, bool SE = false>
__global__ __launch_bounds__(64 * schur_group(NT)) __attribute__((amdgpu_waves_per_eu(2, 2))) void schur_kernel(
    DevProblem P, const CamPre* __restrict__ cps, const double* __restrict__ intr,
    const double* __restrict__ X, double radius, unsigned long long* __restrict__ stamps) {
    constexpr int IW = kIW<CM>;   // tile rows (and F columns) of an intrinsics block
    // intrinsics parameters with a Jacobian column: SNAVELY's 4th double is not one
    constexpr int NK = CM == SFM_CAM_SNAVELY ? 3 : IW;
    unsigned long long tacc[6] = {0, 0, 0, 0, 0, 0}, tprev = 0;
    if (stamps) tprev = stamp();
#define SFM_STAMP(k)                                      \
    if (stamps) {                                         \
        const unsigned long long tn_ = stamp();           \
        tacc[k] += tn_ - tprev;                           \
        tprev = tn_;                                      \
    }
    // LDS strides padded against bank conflicts (MI355X_MICROARCH.md §LDS):
    // panel rows 4 doubles past the tile width put the 12 (point, axis) rows
    // that the intrinsics pass updates at one column on distinct banks, and
    // 14-double observation rows spread ds_write_b128 lane groups.
    constexpr int kPK = 4 * ((3 * SP + 3) / 4), kPR = 16 * NT, kPS = kPR + 4;
    // per-observation rows use odd strides (in doubles): a wave's ds_*_b64 at
    // lane-strided rows then hits 32 distinct bank pairs (even strides of 4,
    // 6, 10 doubles were 2- to 4-way bank conflicts, SQ_LDS_BANK_CONFLICT)
    // pinhole: the 4 nonzeros of J_intr; SNAVELY / RADIAL3: both rows of every
    // parameter column (2 NK values)
    constexpr int kOb = CM == SFM_CAM_PINHOLE ? 5 : 2 * NK + 1;
    constexpr int kNTiles = NT * (NT + 1) / 2;
    constexpr int kComb = 5;                    // tiles per round of the group's tile sum
    // each wave's own LDS; its space also carries the wave's tiles to wave 0
    // at the end (kComb 16x16 tiles per round)
    struct WaveLds {
        double panel[kPK][kPS];                 // [k][row]
        double wcol[NT == 4 ? kPK : 1];         // NT = 4: w = L^-1 g_E per panel column
        double ob[SO][kOb];                     // J_intr nonzeros (scaled) | pad
        // per observation: Jx'Jx (6) | Jx'f (3) until the per-point sums, then
        // M = Jx L^-T (6) from phase B on (obm: the same rows)
        double vs[SO][9];
        double vsum[SP][10];                    // per point: V (6) | g_E (3)
        int orow[SO];                           // tile row of the obs' intrinsics block
        int cpoff[kChunkPts + 1];               // chunk point offsets, relative to obs_begin
    };
    union WaveU {
        WaveLds w;
        double comb[kComb * 256 + 64];          // kComb tiles + the NT = 4 -Zw column
    };
    static_assert(sizeof(WaveLds) >= sizeof(double) * (kComb * 256 + 64), "tile hand-over space");
    constexpr int GW = schur_group(NT);         // waves (chunks) per group
    __shared__ WaveU wl[GW];
    // group-level staging: every camera / intrinsics block the group touches
    __shared__ CamPreL scp[kCamSlots];
    __shared__ double csc[kCamSlots][6];        // camera column scales (0: constant image)
    __shared__ double isc[kIntrSlots][2 * IW];  // intrinsics | their column scales
    __shared__ int crow[kCamSlots], irow[kIntrSlots];
    // wave-uniform (scalar): the LDS bases and chunk fields below stay in SGPRs
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, grp = blockIdx.x;
    const int c0 = P.group_off[grp], n_sub = P.group_off[grp + 1] - c0;
    const int c = c0 + (wave < n_sub ? wave : 0);   // this wave's chunk (a wave past the group's chunks idles)
    const ChunkDesc& cd = P.chunks[c];
    WaveLds& W = wl[wave].w;
    double (&panel)[kPK][kPS] = W.panel;
    double (&wcol)[NT == 4 ? kPK : 1] = W.wcol;
    double (&ob)[SO][kOb] = W.ob;
    double (&vs)[SO][9] = W.vs;
    double (&vsum)[SP][10] = W.vsum;
    double (*const obm)[9] = vs;
    int (&orow)[SO] = W.orow;
    int (&cpoff)[kChunkPts + 1] = W.cpoff;
    const int pb = cd.pt_begin, np = wave < n_sub ? cd.pt_end - pb : 0, ob0 = cd.obs_begin;
    // read once: a ChunkDesc load inside the batch loop would be waited on
    // with the in-order counter, i.e. together with the next batch's prefetch
    const bool one_intr = cd.n_intr == 1;
    const double inv_radius = 1.0 / radius;   // LM diagonal D^2 = clamp(diag) / radius (as step_kernel)

    for (int e = lane; e <= np; e += 64) cpoff[e] = P.pt_off[pb + e] - ob0;
    {   // the group's staging, by all its waves
        constexpr int kCpW = sizeof(CamPre) / 8;
        for (int e = threadIdx.x; e < cd.n_cams * kCpW; e += 64 * GW) {
            const int t = e / kCpW;
            reinterpret_cast<double*>(&scp[t].cp)[e - t * kCpW] =
                reinterpret_cast<const double*>(&cps[cd.cam_img[t]])[e - t * kCpW];
        }
        for (int e = threadIdx.x; e < cd.n_cams * 6; e += 64 * GW) {
            const int t = e / 6, col = cd.cam_col[t];
            csc[t][e - 6 * t] = col >= 0 ? P.scaleF[col + e - 6 * t] : 0.0;
        }
        if (threadIdx.x < cd.n_cams) crow[threadIdx.x] = cd.cam_row[threadIdx.x];
        if (threadIdx.x < IW * cd.n_intr) {
            const int t = threadIdx.x / IW, k = threadIdx.x - IW * t;
            isc[t][k] = intr[IW * cd.intr_id[t] + k];
            isc[t][IW + k] = P.scaleF[cd.intr_col[t] + k];
        }
        if (threadIdx.x < cd.n_intr) irow[threadIdx.x] = cd.intr_row[threadIdx.x];
    }

    v4d acc[kNTiles];
#pragma unroll
    for (int q = 0; q < kNTiles; ++q) acc[q] = v4d{0.0, 0.0, 0.0, 0.0};
    double wacc = 0.0;   // NT = 4: -(Z w)[lane]

    double xn2 = 0.0, gmx = 0.0;
    __syncthreads();
    // A batch's observation stream (uv, slot) and point data (X, column scale)
    // are fetched one batch ahead, so their HBM latency overlaps the current
    // batch's compute instead of opening every batch.
    struct BatchIn {
        int npts, slot, pl;
        double u0, u1, Xp[3], sE[3];
    };
    auto fetch = [&](int q0, BatchIn& in) {
        in.npts = q0 < np ? batch_points<SP, SO>(cpoff, q0, np) : 0;
        in.slot = 0; in.pl = 0; in.u0 = 0.0; in.u1 = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) { in.Xp[k] = 0.0; in.sE[k] = 1.0; }
        const int qo = cpoff[q0 < np ? q0 : np];
        if (lane < cpoff[q0 + in.npts] - qo) {
            const int o = ob0 + qo + lane;
            in.slot = P.obs_slot[o];
            const double2 uv = reinterpret_cast<const double2*>(P.obs_uv)[o];
            in.u0 = uv.x; in.u1 = uv.y;
#pragma unroll
            for (int j = 1; j < SP; ++j) in.pl += (j < in.npts && cpoff[q0 + j] - qo <= lane) ? 1 : 0;
            const size_t g = 3 * (size_t)(pb + q0 + in.pl);   // same address for the point's lanes
#pragma unroll
            for (int k = 0; k < 3; ++k) { in.Xp[k] = X[g + k]; in.sE[k] = P.scaleE[g + k]; }
        }
    };
    BatchIn nx;
    fetch(0, nx);
    // The first batch's loads complete before the loop.  Without this the
    // waitcnt pass merges the loop entry (loads pending in the registers the
    // loop body reads) with the back edge and waits on the counter inside
    // phase A of EVERY batch -- which, the counter being in order, also waits
    // for the next batch's prefetch, so its HBM latency was never hidden.
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    for (int p0 = 0; p0 < np;) {
        const int npts = nx.npts;   // batch [p0, p1)
        if (npts == 0) break;   // a point above SO observations: excluded by the planner
        const int p1 = p0 + npts;
        const int o0 = cpoff[p0], nobs = cpoff[p1] - o0;
        const int slot = nx.slot, pl = nx.pl;
        const double u0 = nx.u0, u1 = nx.u1;
        const double Xp[3] = {nx.Xp[0], nx.Xp[1], nx.Xp[2]};
        double sE[3] = {nx.sE[0], nx.sE[1], nx.sE[2]};
        fetch(p1, nx);
#pragma unroll
        for (int e = lane; e < kPK * kPS / 2; e += 64)
            reinterpret_cast<double2*>(&panel[0][0])[e] = double2{0.0, 0.0};
        if constexpr (NT == 4)
            if (lane < kPK) wcol[lane] = 0.0;   // columns past 3 * npts stay zero
        SFM_STAMP(0)
        // ---- A: observations -> scaled, corrected Jacobians -----------------
        LinT<CM> L;
        const int cs = slot & 255, is = (slot >> 8) & 255;
        if (lane < nobs) linearize<CM, true, true, true>(scp[cs].cp, &isc[is][0], Xp, u0, u1, P.huber_a, L);
        if constexpr (SE) {
            // column norms of the point's unscaled Jx, in observation and row
            // order (as point_scale_kernel): raw Jx staged in obm (free until B)
            if (lane < nobs) {
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int a = 0; a < 3; ++a) obm[lane][3 * r + a] = L.Jx[r][a];
            }
            wsync();
            if (lane < 3 * npts) {
                const int pt = lane / 3, a = lane - 3 * pt;
                const int q0 = cpoff[p0 + pt] - o0, q1 = cpoff[p0 + pt + 1] - o0;
                double cn = 0.0;
                for (int q = q0; q < q1; ++q) {
                    cn = fma(obm[q][a], obm[q][a], cn);
                    cn = fma(obm[q][3 + a], obm[q][3 + a], cn);
                }
                const double se = 1.0 / (1.0 + sqrt(cn));
                vsum[pt][a] = se;   // vsum is rewritten after phase A
                P.scaleE[3 * (size_t)(pb + p0 + pt) + a] = se;
            }
            wsync();
            if (lane < nobs) {
#pragma unroll
                for (int a = 0; a < 3; ++a) sE[a] = vsum[pl][a];
            }
            wsync();   // vsum is reused by the per-point sums below
        }
        if (lane < nobs) {
#pragma unroll
            for (int r = 0; r < 2; ++r) {
#pragma unroll
                for (int a = 0; a < 6; ++a) L.Jc[r][a] *= csc[cs][a];
#pragma unroll
                for (int a = 0; a < 3; ++a) L.Jx[r][a] *= sE[a];
            }
            // this observation's share of its point's V = Jx'Jx and g_E = Jx'f
            double cv[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};   // V00 V10 V11 V20 V21 V22 | b0 b1 b2
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const double j0 = L.Jx[r][0], j1 = L.Jx[r][1], j2 = L.Jx[r][2], fr = L.f[r];
                cv[0] += j0 * j0; cv[1] += j1 * j0; cv[2] += j1 * j1;
                cv[3] += j2 * j0; cv[4] += j2 * j1; cv[5] += j2 * j2;
                cv[6] += j0 * fr; cv[7] += j1 * fr; cv[8] += j2 * fr;
            }
#pragma unroll
            for (int e = 0; e < 9; ++e) vs[lane][e] = cv[e];
            // J_intr rows are [x s, 0, s, 0] and [0, y s, 0, s]: keep the 4 nonzeros
            if constexpr (CM != SFM_CAM_PINHOLE) {
                // both rows of the parameter columns (SNAVELY f, l1, l2: column 3
                // is not a parameter; RADIAL3 f, ppx, ppy, k1, k2, k3)
#pragma unroll
                for (int k = 0; k < NK; ++k) {
                    ob[lane][2 * k] = L.Ji[0][k] * isc[is][IW + k];
                    ob[lane][2 * k + 1] = L.Ji[1][k] * isc[is][IW + k];
                }
            } else {
                ob[lane][0] = L.Ji[0][0] * isc[is][4];
                ob[lane][1] = L.Ji[1][1] * isc[is][5];
                ob[lane][2] = L.Ji[0][2] * isc[is][6];
                ob[lane][3] = L.Ji[1][3] * isc[is][7];
            }
            orow[lane] = irow[is];
        }
        wsync();
        // per-point sums in observation order, one lane per (point, entry)
        if (lane < 9 * npts) {
            const int pt = lane / 9, e = lane - 9 * pt;
            const int q0 = cpoff[p0 + pt] - o0, q1 = cpoff[p0 + pt + 1] - o0;
            double acc = 0.0;
            int q = q0;
            for (; q + 4 <= q1; q += 4) {   // loads in flight together, adds in order
                const double v0 = vs[q][e], v1 = vs[q + 1][e], v2 = vs[q + 2][e], v3 = vs[q + 3][e];
                acc += v0; acc += v1; acc += v2; acc += v3;
            }
            for (; q < q1; ++q) acc += vs[q][e];
            vsum[pt][e] = acc;
        }
        wsync();
        SFM_STAMP(1)
        // ---- B: every observation lane takes its point's V + D^2 and g_E (the
        // per-point sums above: identical on all lanes of the point), factors
        // it, and goes on to M = Jx L^-T and the camera rows of Z ----
        if (lane < nobs) {
            const int q0 = cpoff[p0 + pl] - o0;
            double V[6], b[3];   // V00 V10 V11 V20 V21 V22
#pragma unroll
            for (int e = 0; e < 6; ++e) V[e] = vsum[pl][e];
#pragma unroll
            for (int e = 0; e < 3; ++e) b[e] = vsum[pl][6 + e];
            const bool first = lane == q0;
            if (first) {   // gradient / norm bookkeeping at x (used after a relinearisation)
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    const double g = b[a] * rcp_nr(sE[a]);
                    xn2 += Xp[a] * Xp[a];
                    gmx = fmax(gmx, fabs(Xp[a] - (Xp[a] - g)));
                }
            }
            const int di[3] = {0, 2, 5};
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                V[di[a]] += point_d2(P, V[di[a]], inv_radius);
            }
            const double i00 = rsqrt_nr(V[0]);
            const double l10 = V[1] * i00, l20 = V[3] * i00;
            const double i11 = rsqrt_nr(V[2] - l10 * l10);
            const double l21 = (V[4] - l20 * l10) * i11;
            const double i22 = rsqrt_nr(V[5] - l20 * l20 - l21 * l21);
            const double i10 = -l10 * i00 * i11, i21 = -l21 * i11 * i22;
            const double i20 = -(l20 * i00 + l21 * i10) * i22;
            if (first) {
                const double w3[3] = {i00 * b[0], i10 * b[0] + i11 * b[1], i20 * b[0] + i21 * b[1] + i22 * b[2]};
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    if constexpr (NT == 5) panel[3 * pl + a][kTileWRow % kPR] = w3[a];
                    else wcol[3 * pl + a] = w3[a];
                }
            }
            double M[2][3];
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                M[r][0] = L.Jx[r][0] * i00;
                M[r][1] = L.Jx[r][0] * i10 + L.Jx[r][1] * i11;
                M[r][2] = L.Jx[r][0] * i20 + L.Jx[r][1] * i21 + L.Jx[r][2] * i22;
            }
            const int row = crow[cs];
            if (row >= 0) {
#pragma unroll
                for (int a = 0; a < 3; ++a)
#pragma unroll
                    for (int k = 0; k < 6; ++k)
                        panel[3 * pl + a][row + k] = L.Jc[0][k] * M[0][a] + L.Jc[1][k] * M[1][a];
            }
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int a = 0; a < 3; ++a) obm[lane][3 * r + a] = M[r][a];
        }
        wsync();
        SFM_STAMP(2)
        // ---- C2: intrinsics rows, ordered per point ---------------------------
        // (register sums per run of observations sharing an intrinsics block)
        // One intrinsics block in the chunk (shared intrinsics, as C4 and the
        // SequentialActuator's single camera): every observation has the same
        // row, so the sums run without the run-boundary test (same fma order,
        // same bits as the general loops below).
        if (one_intr) {
            constexpr int NZ = 3 * NK;   // (axis, column) sums per point
            const int row = irow[0];
            for (int e = lane; e < NZ * npts; e += 64) {
                const int pt = e / NZ, rem = e - NZ * pt, a = rem / NK, k = rem - NK * a;
                const int q0 = cpoff[p0 + pt] - o0, q1 = cpoff[p0 + pt + 1] - o0;
                double z = 0.0;
                int q = q0;
                if constexpr (CM == SFM_CAM_PINHOLE) {
                    // z_k = sum_q Ji[q][k] M[q][k & 1][a]
                    const int mo = 3 * (k & 1) + a;
                    for (; q + 4 <= q1; q += 4) {
                        double jv[4], mv[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j) { jv[j] = ob[q + j][k]; mv[j] = obm[q + j][mo]; }
#pragma unroll
                        for (int j = 0; j < 4; ++j) z = fma(jv[j], mv[j], z);
                    }
                    for (; q < q1; ++q) z = fma(ob[q][k], obm[q][mo], z);
                } else {
                    for (; q + 2 <= q1; q += 2) {
                        double jv[4], mv[4];
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            jv[2 * j] = ob[q + j][2 * k]; jv[2 * j + 1] = ob[q + j][2 * k + 1];
                            mv[2 * j] = obm[q + j][a]; mv[2 * j + 1] = obm[q + j][3 + a];
                        }
#pragma unroll
                        for (int j = 0; j < 4; ++j) z = fma(jv[j], mv[j], z);
                    }
                    for (; q < q1; ++q) {
                        z = fma(ob[q][2 * k], obm[q][a], z);
                        z = fma(ob[q][2 * k + 1], obm[q][3 + a], z);
                    }
                }
                panel[3 * pt + a][row + k] += z;
            }
        } else if constexpr (CM != SFM_CAM_PINHOLE) {
            // one lane per (point, axis, intrinsics column k < NK):
            // z_k = sum_q Ji[q][0][k] M[q][0][a] + Ji[q][1][k] M[q][1][a]
            for (int e = lane; e < 3 * NK * npts; e += 64) {
                const int pt = e / (3 * NK), rem = e - 3 * NK * pt, a = rem / NK, k = rem - NK * a;
                const int q0 = cpoff[p0 + pt] - o0, q1 = cpoff[p0 + pt + 1] - o0;
                int row = orow[q0];
                double z = 0.0;
                for (int q = q0; q < q1; ++q) {
                    const int rq = orow[q];
                    if (rq != row) {
                        panel[3 * pt + a][row + k] += z;
                        z = 0.0;
                        row = rq;
                    }
                    z = fma(ob[q][2 * k], obm[q][a], z);
                    z = fma(ob[q][2 * k + 1], obm[q][3 + a], z);
                }
                panel[3 * pt + a][row + k] += z;
            }
        } else if constexpr (12 * SP <= 64) {
            // one lane per (point, axis, intrinsics column): z_k = sum_q Ji[q][k] M[q][k & 1][a]
            if (lane < 12 * npts) {
                const int pt = lane / 12, rem = lane - 12 * pt, a = rem >> 2, k = rem & 3;
                const int mo = 3 * (k & 1) + a;
                const int q0 = cpoff[p0 + pt] - o0, q1 = cpoff[p0 + pt + 1] - o0;
                int row = orow[q0];
                double z = 0.0;
                auto step = [&](int rq, double jv, double mv) {
                    if (rq != row) {
                        panel[3 * pt + a][row + k] += z;
                        z = 0.0;
                        row = rq;
                    }
                    z = fma(jv, mv, z);
                };
                int q = q0;
                for (; q + 4 <= q1; q += 4) {   // operands of 4 observations loaded together
                    int rq[4];
                    double jv[4], mv[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) { rq[j] = orow[q + j]; jv[j] = ob[q + j][k]; mv[j] = obm[q + j][mo]; }
#pragma unroll
                    for (int j = 0; j < 4; ++j) step(rq[j], jv[j], mv[j]);
                }
                for (; q < q1; ++q) step(orow[q], ob[q][k], obm[q][mo]);
                panel[3 * pt + a][row + k] += z;
            }
        } else if (lane < 3 * npts) {
            const int pt = lane / 3, a = lane - 3 * pt;
            const int q0 = cpoff[p0 + pt] - o0, q1 = cpoff[p0 + pt + 1] - o0;
            int row = orow[q0];
            double z0 = 0.0, z1 = 0.0, z2 = 0.0, z3 = 0.0;
            for (int q = q0; q < q1; ++q) {
                const int rq = orow[q];
                if (rq != row) {
                    panel[3 * pt + a][row + 0] += z0; panel[3 * pt + a][row + 1] += z1;
                    panel[3 * pt + a][row + 2] += z2; panel[3 * pt + a][row + 3] += z3;
                    z0 = z1 = z2 = z3 = 0.0;
                    row = rq;
                }
                const double m0 = obm[q][a], m1 = obm[q][3 + a];
                z0 += ob[q][0] * m0;
                z1 += ob[q][1] * m1;
                z2 += ob[q][2] * m0;
                z3 += ob[q][3] * m1;
            }
            panel[3 * pt + a][row + 0] += z0; panel[3 * pt + a][row + 1] += z1;
            panel[3 * pt + a][row + 2] += z2; panel[3 * pt + a][row + 3] += z3;
        }
        wsync();
        SFM_STAMP(3)
        // ---- D: tile += panel panel' on the fp64 MFMA -------------------------
        // all operands first (padding columns are zero), then the MFMAs
        const int kk = lane >> 4, ii = lane & 15;
        constexpr int kKs = kPK / 4;
        double op[kKs][NT];
#pragma unroll
        for (int ks = 0; ks < kKs; ++ks)
#pragma unroll
            for (int t = 0; t < NT; ++t) op[ks][t] = panel[4 * ks + kk][16 * t + ii];
#pragma unroll
        for (int ks = 0; ks < kKs; ++ks)
#pragma unroll
            for (int q = 0; q < kNTiles; ++q)
                acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(op[ks][kTi[q]], op[ks][kTj[q]], acc[q], 0, 0, 0);
        if constexpr (NT == 4) {
#pragma unroll
            for (int k = 0; k < kPK; ++k) wacc += panel[k][lane] * wcol[k];
        }
        wsync();
        SFM_STAMP(4)
        p0 = p1;
    }
    // ---- the group's tile: waves 1.. hand their accumulators to wave 0
    // through their own LDS, kComb 16x16 tiles per round, added in wave order;
    // wave 0 writes the negated tile, its lower 16x16 tiles only (the gather
    // reads upper blocks at their symmetric partner, FlatTerm modes)
    __syncthreads();   // every wave is past its batch loop: its LDS is free
    double* out = P.tiles + (size_t)grp * kTileR * kTileR;
#pragma unroll
    for (int q0 = 0; q0 < kNTiles; q0 += kComb) {
        if (wave > 0 && wave < n_sub) {
            double* cb = wl[wave].comb;
#pragma unroll
            for (int q = q0; q < q0 + kComb && q < kNTiles; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) cb[(q - q0) * 256 + r * 64 + lane] = acc[q][r];
            if (NT == 4 && q0 == 0) cb[kComb * 256 + lane] = wacc;
        }
        __syncthreads();
        if (wave == 0) {
            for (int w2 = 1; w2 < n_sub; ++w2) {
                const double* cb = wl[w2].comb;
#pragma unroll
                for (int q = q0; q < q0 + kComb && q < kNTiles; ++q)
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[q][r] += cb[(q - q0) * 256 + r * 64 + lane];
                if (NT == 4 && q0 == 0) wacc += cb[kComb * 256 + lane];
            }
#pragma unroll
            for (int q = q0; q < q0 + kComb && q < kNTiles; ++q) {
                const int ti = kTi[q], tj = kTj[q];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 16 * ti + (lane >> 4) + 4 * r, col = 16 * tj + (lane & 15);
                    out[row * kTileR + col] = -acc[q][r];
                }
            }
            if (NT == 4 && q0 == 0) out[kTileWRow * kTileR + lane] = -wacc;
        }
        if (q0 + kComb < kNTiles) __syncthreads();   // wave 0 has read this round
    }
    // ---- point partials of this wave's chunk (fixed-order wave reduction) ----
    double s1[1] = {xn2};
    wave_sum(s1);
    const double m1 = wave_max(gmx);
    if (lane == 0 && wave < n_sub) {
        P.part_s[2 * (size_t)c] = s1[0];
        P.part_s[2 * (size_t)c + 1] = m1;
    }
    SFM_STAMP(5)
    if (stamps && lane == 0 && wave < n_sub)
        for (int k = 0; k < 6; ++k) stamps[6 * (size_t)c + k] = tacc[k];
#undef SFM_STAMP
}

// ---------------------------------------------------------------------------
// static gather-reduce: one wave per target block
// ---------------------------------------------------------------------------
__device__ __forceinline__ double term_value(const DevProblem& P, const FlatTerm& q, int r, int cc) {
    // all three index forms computed and selected without branches, so the
    // reduce loops keep a batch of term loads in flight
    const int t = q.rs;   // kFlatSym: the origin's offset within the tile
    const int R = t / kTileR + r, C = t % kTileR + cc;
    const int64_t i_rows = q.off + (int64_t)r * q.rs + cc;
    const int64_t i_trans = q.off + (int64_t)cc * kTileR + r;
    const int64_t i_sym = q.off - t + (R >= C ? R * kTileR + C : C * kTileR + R);
    const int64_t idx = q.mode == kFlatRows ? i_rows : q.mode == kFlatTrans ? i_trans : i_sym;
    return (double)q.sign * P.src[idx];
}

// s += term k, k + step, ... (k < end), in that order.  Batches of kRB: the
// descriptors first, then the data they address; the next batch's
// descriptors are issued behind this batch's data loads, and the tail batch
// is masked (clamped loads, masked adds) -- so a lane's chain is about one
// global round trip per batch instead of two, and a few terms past a whole
// batch no longer run one dependent round trip pair each.  The additions are
// those of the term-at-a-time loop, in its order (same bits).  kRB = 8
// (profiles/r05/r_red, same box): reduce 34.2 -> 34.9 us at C4, 20.5 ->
// 19.0 at rank 0 of N = 8 (2836-2846 -> 2854-2856 LM-iters/s); 16 took the
// kernel to 208 VGPRs, 2 waves per SIMD, and C4's reduce to 49.5 us.
#ifndef SFM_REDUCE_BATCH
#define SFM_REDUCE_BATCH 8
#endif
constexpr int kRB = SFM_REDUCE_BATCH;   // terms per batch (A/B builds only)
__device__ __forceinline__ double sum_terms(const DevProblem& P, int k, int step, int end, int r, int cc) {
    double s = 0.0;
    if (k >= end) return s;
    const int k_safe = k;
    FlatTerm d[kRB];
    auto ld_desc = [&](int k0) {
#pragma unroll
        for (int j = 0; j < kRB; ++j) {
            const int kj = k0 + j * step;
            d[j] = P.terms[kj < end ? kj : k_safe];
        }
    };
    ld_desc(k);
    for (; k < end; k += kRB * step) {
        double v[kRB];
#pragma unroll
        for (int j = 0; j < kRB; ++j) v[j] = term_value(P, d[j], r, cc);
        if (k + kRB * step < end) ld_desc(k + kRB * step);
#pragma unroll
        for (int j = 0; j < kRB; ++j)
            if (k + j * step < end) s += v[j];
    }
    return s;
}

__device__ __forceinline__ double* target_base(const DevProblem& P, int kind) {
    switch (kind) {
        case 0: return P.Sband;
        case 1: return P.Sarrow;
        case 2: return P.Scorner;
        case 3: return P.rhs;
        case 4: return P.bF;
        case 5: return P.cnF;
        default: return P.Sdense;
    }
}

// Longer term lists are summed by a whole workgroup (256 parallel chains);
// shorter ones by one lane per element.  A camera's band blocks collect
// ~2 * points-per-camera / chunk-points terms (about 80 at C4), the
// intrinsics corner one per chunk (thousands).
constexpr int kLongTerms = 256;

// vectors_only (iteration 0, before the Jacobi scales): bF and cnF only
__device__ __forceinline__ bool skip_kind(int kind, int vectors_only) {
    return vectors_only && kind != kDstBF && kind != kDstCnF;
}

// P.red_waves (1, 2 or 4) waves per target: wave w of a target sums its
// lane groups' terms w, w + W, ... (in units of G), and the partials are added
// in (wave, group) order -- fixed, so deterministic.  More waves per target
// shorten the chain of dependent term loads where targets collect many terms
// (a landmark shard at N = 8 has ~30-point chunks, so ~170 tile terms per
// band block against ~80 at N = 1).
template <bool FUSED>
__device__ void reduce_segment(const DevProblem& P, int vectors_only, int sg);

// n_short_blocks: the short targets' workgroups; FUSED: every workgroup past
// them is one segment of a long target (reduce_segment<true>), so the whole
// reduce is one launch instead of three
// zero_first: the first workgroup of the zero list (world > 1: the blocks
// other shards write, cleared before the all-reduce; 16 per workgroup, every
// kind, also in the vectors-only pass)
template <bool FUSED>
__global__ __launch_bounds__(256) void reduce_kernel(DevProblem P, int vectors_only, int n_short_blocks,
                                                     int zero_first) {
    if ((int)blockIdx.x >= zero_first) {
        const int wave = threadIdx.x >> 6, e = threadIdx.x & 63;
        for (int q = 0; q < 4; ++q) {
            const int z = ((int)blockIdx.x - zero_first) * 16 + wave * 4 + q;
            if (z >= P.n_zero) break;
            const ReduceTarget T = P.targets[P.n_targets + z];
            const int E = T.rows * T.cols;
            if (e < E) {
                const int r = e / T.cols, cc = e % T.cols;
                target_base(P, T.dst_kind)[T.dst + (T.cols == 1 ? r : r * T.ld + cc)] = 0.0;
            }
        }
        return;
    }
    if (FUSED && (int)blockIdx.x >= n_short_blocks) {
        reduce_segment<true>(P, vectors_only, blockIdx.x - n_short_blocks);
        return;
    }
    const int W = P.red_waves, wave = threadIdx.x >> 6, e = threadIdx.x & 63;
    const int t = blockIdx.x * (4 / W) + wave / W, ws = wave - (wave / W) * W;
    __shared__ double part[4][64];
    bool live = t < P.n_targets;
    ReduceTarget T{};
    if (live) {
        T = P.targets[t];
        live = !skip_kind(T.dst_kind, vectors_only) && T.c_end - T.c_begin <= kLongTerms;
    }
    // G = 64 / E lane groups of the target's E elements: group g sums terms
    // g, g + G, ... (a 6-vector target keeps 60 lanes busy instead of 6)
    const int E = live ? T.rows * T.cols : 64, G = 64 / E, g = e / E, el = e - g * E;
    const int r = live ? el / T.cols : 0, cc = live ? el % T.cols : 0;
    // a target is a chain of dependent global round trips (term descriptor,
    // then data): sum_terms keeps 16 terms and the next 16 descriptors in flight
    double s = 0.0;
    if (live && g < G) s = sum_terms(P, T.c_begin + ws * G + g, G * W, T.c_end, r, cc);
    if (W > 1) {   // (uniform over the launch: every wave reaches the barrier)
        part[wave][e] = s;
        __syncthreads();
        if (!live || ws != 0 || g != 0) return;
        s = 0.0;
        for (int w = 0; w < W; ++w)
            for (int q = 0; q < G; ++q) s += part[wave + w][q * E + el];
    } else if (G > 1) {
        part[wave][e] = s;
        wsync();
        if (!live || g != 0) return;
        s = 0.0;
        for (int q = 0; q < G; ++q) s += part[wave][q * E + el];
    } else if (!live || g != 0) {   // (G = 1: lanes past the E elements)
        return;
    }
    const bool vec = T.cols == 1;
    target_base(P, T.dst_kind)[T.dst + (vec ? r : r * T.ld + cc)] = s;
}

// Long targets, pass 1: one workgroup per kReduceSeg-term segment, one term
// per thread (every element of the block, <= 36, in registers); the 256
// partial blocks are combined by xor-butterflies and wave order (fixed).
// (one workgroup: segment sg of its long target, partial into lpart[sg];
// FUSED: stored write-through, and the target's last segment to finish adds
// the partials in segment order -- the same sum as reduce_long_kernel)
template <bool FUSED>
__device__ __forceinline__ void reduce_segment(const DevProblem& P, int vectors_only, int sg) {
    const int j = P.lseg[2 * sg], k0 = P.lseg[2 * sg + 1];
    const ReduceTarget T = P.targets[P.long_targets[j]];
    if (skip_kind(T.dst_kind, vectors_only)) return;   // (uniform over the workgroup)
    // each wave a quarter of the segment, in G = 64 / E lane groups of the
    // target's E elements (as reduce_kernel); partials added in (wave, group)
    // order, fixed
    const int E = T.rows * T.cols, G = 64 / E;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane / E, el = lane - g * E;
    constexpr int kQ = kReduceSeg / 4;
    const int q0 = k0 + wave * kQ, q1 = min(min(k0 + kReduceSeg, (int)T.c_end), q0 + kQ);
    double s = 0.0;
    if (g < G) s = sum_terms(P, q0 + g, G, q1, el / T.cols, el % T.cols);
    __shared__ double part[4][64];
    __shared__ int last;
    part[wave][lane] = s;
    __syncthreads();
    if ((int)threadIdx.x < E) {
        const int t = threadIdx.x;
        double tot = 0.0;
        for (int w = 0; w < 4; ++w)
            for (int q = 0; q < G; ++q) tot += part[w][q * E + t];
        if (FUSED) st_wt64(P.lpart + (size_t)sg * 36 + t, tot);
        else P.lpart[(size_t)sg * 36 + t] = tot;
    }
    if (!FUSED) return;
    // the partial is drained before the ticket; the last arriver reads every
    // partial of the target write-through (no fences: the counter form)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int s0 = P.lseg_off[j], s1 = P.lseg_off[j + 1];
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add((gu32_t*)(P.lcount + j), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               (unsigned)(s1 - s0 - 1);
    __syncthreads();
    if (!last) return;
    if ((int)threadIdx.x < E) {
        const int e = threadIdx.x;
        double t = 0.0;
#pragma unroll 8
        for (int q = s0; q < s1; ++q) t += ld_wt64(P.lpart + (size_t)q * 36 + e);
        const int r = e / T.cols, cc = e % T.cols;
        target_base(P, T.dst_kind)[T.dst + (T.cols == 1 ? r : r * T.ld + cc)] = t;
    }
    if (threadIdx.x == 0)   // ready for the next launch (stream order)
        __hip_atomic_store((gu32_t*)(P.lcount + j), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void reduce_seg_kernel(DevProblem P, int vectors_only) {
    reduce_segment<false>(P, vectors_only, blockIdx.x);
}

// pass 2: segment partials added in segment order
__global__ __launch_bounds__(64) void reduce_long_kernel(DevProblem P, int vectors_only) {
    const int j = blockIdx.x;
    const ReduceTarget T = P.targets[P.long_targets[j]];
    if (skip_kind(T.dst_kind, vectors_only)) return;
    const int E = T.rows * T.cols, e = threadIdx.x;
    if (e >= E) return;
    double t = 0.0;
#pragma unroll 8
    for (int sg = P.lseg_off[j]; sg < P.lseg_off[j + 1]; ++sg) t += P.lpart[(size_t)sg * 36 + e];
    const int r = e / T.cols, cc = e % T.cols;
    target_base(P, T.dst_kind)[T.dst + (T.cols == 1 ? r : r * T.ld + cc)] = t;
}

// ---------------------------------------------------------------------------
// RCS solve: block-banded (6x6 blocks, half-bandwidth D) Cholesky with a dense
// intrinsics arrow, over a circular window of D+1 block rows.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double lm2(const DevProblem& P, int64_t col, double radius) {
    const double lm = sqrt(clampd(P.cnF[col], P.min_diag, P.max_diag) / radius);
    return lm * lm;
}

__device__ bool chol_inplace(double* A, int n, int ld) {  // lower, serial
    bool ok = true;
    for (int j = 0; j < n; ++j) {
        double s = A[j * ld + j];
        for (int k = 0; k < j; ++k) s -= A[j * ld + k] * A[j * ld + k];
        if (!(s > 0.0)) ok = false;
        const double d = sqrt(s);
        A[j * ld + j] = d;
        const double id = 1.0 / d;
        for (int i = j + 1; i < n; ++i) {
            double t = A[i * ld + j];
            for (int k = 0; k < j; ++k) t -= A[i * ld + k] * A[j * ld + k];
            A[i * ld + j] = t * id;
        }
    }
    return ok;
}

__global__ __launch_bounds__(256) void solve_kernel(DevProblem P, double radius, int use_lds) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int ncam = P.ncam, nintr = P.nintr, D = P.D, Dp = D + 1;
    const int tid = threadIdx.x;
    // LDS: [fail (2 doubles) | YW (Dp x 6) | window if it fits]; else window in HBM
    double* failp = lds;
    double* YW = lds + 2;                                   // [Dp][6], always LDS
    double* W = use_lds ? lds + 2 + (size_t)Dp * 6 : P.Wglobal;
    double* WA = W + (size_t)Dp * Dp * 36;                // [nintr][Dp][24]
    double* WC = WA + (size_t)nintr * Dp * 24;             // [4nintr][4nintr]
    double* WR = WC + (size_t)16 * nintr * nintr;          // [Dp][6]
    double* WRA = WR + (size_t)Dp * 6;                     // [4nintr]
    int fail_local = 0;
    const int na4 = 4 * nintr;

    auto Wb = [&](int i, int d) { return W + ((size_t)(i % Dp) * Dp + d) * 36; };
    auto WAb = [&](int k, int j) { return WA + ((size_t)k * Dp + (j % Dp)) * 24; };

    auto load_row = [&](int i) {
        const int dm = min(D, i);
        for (int e = tid; e < (dm + 1) * 36; e += 256) {
            const int d = e / 36, q = e % 36;
            double v = P.Sband[((size_t)i * Dp + d) * 36 + q];
            if (d == 0 && q % 7 == 0) v += lm2(P, 6LL * i + q / 7, radius);
            Wb(i, d)[q] = v;
        }
        for (int e = tid; e < nintr * 24; e += 256) {
            const int k = e / 24, q = e % 24;
            WAb(k, i)[q] = P.Sarrow[((size_t)k * ncam + i) * 24 + q];
        }
        if (tid < 6) WR[(i % Dp) * 6 + tid] = P.rhs[6LL * i + tid];
    };
    // corner (dense 4nintr x 4nintr from 4x4 blocks) and arrow rhs
    for (int e = tid; e < na4 * na4; e += 256) {
        const int rr = e / na4, cc = e % na4;
        double v = P.Scorner[(((size_t)(rr / 4) * nintr + cc / 4) * 16) + (rr % 4) * 4 + cc % 4];
        if (rr == cc) v += lm2(P, P.nb + rr, radius);
        WC[e] = v;
    }
    if (tid < na4) WRA[tid] = P.rhs[P.nb + tid];
    for (int i = 0; i < min(Dp, ncam); ++i) load_row(i);
    __syncthreads();

    for (int j = 0; j < ncam; ++j) {
        const int dm = min(D, ncam - 1 - j);
        // (a) factor the diagonal block; forward-substitute its rhs
        if (tid == 0) {
            double* Ljj = Wb(j, 0);
            if (!chol_inplace(Ljj, 6, 6)) fail_local = 1;
            double* z = WR + (j % Dp) * 6;
            for (int r = 0; r < 6; ++r) {
                double s = z[r];
                for (int k = 0; k < r; ++k) s -= Ljj[r * 6 + k] * z[k];
                z[r] = s / Ljj[r * 6 + r];
            }
        }
        __syncthreads();
        // (b) TRSM: rows of blocks (j+d, j) and arrow rows: X L_jj' = S
        {
            const double* Ljj = Wb(j, 0);
            const int nrows = 6 * dm + na4;
            for (int t = tid; t < nrows; t += 256) {
                double* row;
                if (t < 6 * dm) row = Wb(j + t / 6 + 1, t / 6 + 1) + (t % 6) * 6;
                else row = WAb((t - 6 * dm) / 4, j) + ((t - 6 * dm) % 4) * 6;
                for (int cc = 0; cc < 6; ++cc) {
                    double s = row[cc];
                    for (int m = 0; m < cc; ++m) s -= row[m] * Ljj[cc * 6 + m];
                    row[cc] = s / Ljj[cc * 6 + cc];
                }
            }
        }
        __syncthreads();
        // (c) trailing updates + rhs updates + write column j out
        {
            const double* z = WR + (j % Dp) * 6;
            const int npair = dm * (dm + 1) / 2;
            const int nb_el = npair * 36, na_el = nintr * dm * 24, nc_el = na4 * na4;
            const int nr_el = 6 * dm + na4;
            const int total = nb_el + na_el + nc_el + nr_el;
            for (int t = tid; t < total; t += 256) {
                if (t < nb_el) {
                    const int q = t / 36, e = t % 36, r = e / 6, cc = e % 6;
                    int di = (int)((1.0 + sqrt(1.0 + 8.0 * q)) * 0.5);
                    while (di * (di - 1) / 2 > q) --di;
                    while ((di + 1) * di / 2 <= q) ++di;
                    const int dk = q - di * (di - 1) / 2 + 1;
                    const double* Li = Wb(j + di, di) + r * 6;
                    const double* Lk = Wb(j + dk, dk) + cc * 6;
                    double s = 0.0;
#pragma unroll
                    for (int m = 0; m < 6; ++m) s += Li[m] * Lk[m];
                    Wb(j + di, di - dk)[e] -= s;
                } else if (t < nb_el + na_el) {
                    const int u = t - nb_el, k = u / (dm * 24), rem = u % (dm * 24);
                    const int dk = rem / 24 + 1, e = rem % 24, r = e / 6, cc = e % 6;
                    const double* La = WAb(k, j) + r * 6;
                    const double* Lk = Wb(j + dk, dk) + cc * 6;
                    double s = 0.0;
#pragma unroll
                    for (int m = 0; m < 6; ++m) s += La[m] * Lk[m];
                    WAb(k, j + dk)[e] -= s;
                } else if (t < nb_el + na_el + nc_el) {
                    const int u = t - nb_el - na_el, rr = u / na4, cc = u % na4;
                    const double* La = WAb(rr / 4, j) + (rr % 4) * 6;
                    const double* Lb = WAb(cc / 4, j) + (cc % 4) * 6;
                    double s = 0.0;
#pragma unroll
                    for (int m = 0; m < 6; ++m) s += La[m] * Lb[m];
                    WC[u] -= s;
                } else {
                    const int u = t - nb_el - na_el - nc_el;
                    if (u < 6 * dm) {
                        const int di = u / 6 + 1, r = u % 6;
                        const double* Li = Wb(j + di, di) + r * 6;
                        double s = 0.0;
#pragma unroll
                        for (int m = 0; m < 6; ++m) s += Li[m] * z[m];
                        WR[((j + di) % Dp) * 6 + r] -= s;
                    } else {
                        const int a = u - 6 * dm;
                        const double* La = WAb(a / 4, j) + (a % 4) * 6;
                        double s = 0.0;
#pragma unroll
                        for (int m = 0; m < 6; ++m) s += La[m] * z[m];
                        WRA[a] -= s;
                    }
                }
            }
            for (int e = tid; e < (dm + 1) * 36; e += 256)
                P.Lcol[((size_t)j * Dp + e / 36) * 36 + e % 36] = Wb(j + e / 36, e / 36)[e % 36];
            for (int e = tid; e < nintr * 24; e += 256)
                P.Larrow[((size_t)j * nintr + e / 24) * 24 + e % 24] = WAb(e / 24, j)[e % 24];
            if (tid < 6) P.zF[6LL * j + tid] = z[tid];
        }
        __syncthreads();
        // (d) slide the window: block row j+Dp takes row j's slot
        if (j + Dp < ncam) load_row(j + Dp);
        __syncthreads();
    }
    // corner: factor, forward, backward
    if (tid == 0) {
        if (na4 > 0 && !chol_inplace(WC, na4, na4)) fail_local = 1;
        for (int r = 0; r < na4; ++r) {
            double s = WRA[r];
            for (int k = 0; k < r; ++k) s -= WC[r * na4 + k] * WRA[k];
            WRA[r] = s / WC[r * na4 + r];
        }
        for (int r = na4 - 1; r >= 0; --r) {
            double s = WRA[r];
            for (int k = r + 1; k < na4; ++k) s -= WC[k * na4 + r] * WRA[k];
            WRA[r] = s / WC[r * na4 + r];
            P.yF[P.nb + r] = WRA[r];
        }
    }
    __syncthreads();
    // back substitution over the band (wave 0)
    if (tid < 64) {
        const int lane = tid;
        for (int j = ncam - 1; j >= 0; --j) {
            const int dm = min(D, ncam - 1 - j);
            double s[6] = {0, 0, 0, 0, 0, 0};
            const int nterm = 6 * dm + na4;
            for (int t = lane; t < nterm; t += 64) {
                const double* Lrow;  // row (c) of the block: L[c][0..5]
                double yv;
                if (t < 6 * dm) {
                    const int d = t / 6 + 1, cc = t % 6;
                    Lrow = P.Lcol + ((size_t)j * Dp + d) * 36 + cc * 6;
                    yv = YW[((j + d) % Dp) * 6 + cc];
                } else {
                    const int a = t - 6 * dm;
                    Lrow = P.Larrow + ((size_t)j * nintr + a / 4) * 24 + (a % 4) * 6;
                    yv = WRA[a];
                }
#pragma unroll
                for (int r = 0; r < 6; ++r) s[r] += Lrow[r] * yv;
            }
            wave_sum(s);
            if (lane == 0) {
                const double* Ljj = P.Lcol + ((size_t)j * Dp) * 36;
                double y[6];
                for (int r = 5; r >= 0; --r) {
                    double v = P.zF[6LL * j + r] - s[r];
                    for (int k = r + 1; k < 6; ++k) v -= Ljj[k * 6 + r] * y[k];
                    y[r] = v / Ljj[r * 6 + r];
                }
                for (int r = 0; r < 6; ++r) {
                    YW[(j % Dp) * 6 + r] = y[r];
                    P.yF[6LL * j + r] = y[r];
                }
            }
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
        }
    }
    __syncthreads();
    (void)failp;
    if (tid == 0) P.scal[kScSolveFail] = fail_local ? 1.0 : 0.0;
}

// ---------------------------------------------------------------------------
// Candidate parameters: one thread per image / intrinsic block.  Active
// columns take x - yF*scaleF (Ceres' x + delta in the unscaled frame),
// inactive (constant) blocks are copied; the candidate CamPre is built inline.
// Per-workgroup partials of |x|^2, |delta|^2 and max|g| over the F columns go
// to part_f and are summed in fixed order by finalize_kernel.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kCandThreads) void cand_kernel(DevProblem P,
                                                            const double* __restrict__ extr,
                                                            const double* __restrict__ intr,
                                                            double* __restrict__ cand_extr,
                                                            double* __restrict__ cand_intr,
                                                            CamPre* __restrict__ cand_cp) {
    const int t = blockIdx.x * kCandThreads + threadIdx.x;
    CandAcc ca;
    auto col = [&](double x, int64_t c) { return cand_col(x, P.yF[c], P.scaleF[c], P.bF[c], ca); };
    if (t < P.n_img) {
        const int c0 = P.img_colc[t];
        double e[6];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const double x = extr[6 * (size_t)t + a];
            e[a] = c0 >= 0 ? col(x, (int64_t)c0 + a) : x;
            cand_extr[6 * (size_t)t + a] = e[a];
        }
        cand_cp[t] = make_campre(e);
    } else if (t < P.n_img + P.n_intr) {
        const int q = t - P.n_img;
        const int c0 = P.intr_col[q];
        // SNAVELY: the 4th double is not a parameter (not moved, not in the norms)
        const int iw = P.iw, na = P.cam_model == SFM_CAM_SNAVELY ? 3 : iw;
        for (int a = 0; a < iw; ++a) {
            const double x = intr[iw * (size_t)q + a];
            cand_intr[iw * (size_t)q + a] = (c0 >= 0 && a < na) ? col(x, (int64_t)c0 + a) : x;
        }
    }
    double v[2] = {ca.x2, ca.d2};
    wave_sum(v);
    const double gm = wave_max(ca.gm);
    constexpr int kW = kCandThreads / 64;
    __shared__ double red[kW][3];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) { red[wave][0] = v[0]; red[wave][1] = v[1]; red[wave][2] = gm; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double r[3] = {0.0, 0.0, 0.0};
        for (int w = 0; w < kW; ++w) { r[0] += red[w][0]; r[1] += red[w][1]; r[2] = fmax(r[2], red[w][2]); }
        for (int k = 0; k < 3; ++k) P.part_f[3 * (size_t)blockIdx.x + k] = r[k];
    }
}

// ---------------------------------------------------------------------------
// per-point back substitution, model cost change, candidate cost
// One workgroup per Schur chunk, SPLIT threads per point (adjacent lanes, each
// taking every SPLIT-th observation; their sums are combined with xor
// shuffles, identical in every lane of the group), at most kStepThreads
// threads.  A landmark shard at N = 8 has short chunks (~30 points, so that
// the Schur pass keeps dividing by N): one thread per point would leave three
// quarters of a 128-thread workgroup idle and each lane a chain of 20
// linearisations.  The chunk's current and candidate cameras, intrinsics, column scales
// and y_F are staged in LDS once, so the per-observation work gathers only the
// measurement.
// ---------------------------------------------------------------------------
constexpr int kStepThreads = 256;
template <int CM, int SPLIT>
__global__ __launch_bounds__(kStepThreads) void step_kernel(DevProblem P, const CamPre* __restrict__ cps,
                                                         const double* __restrict__ intr,
                                                         const CamPre* __restrict__ cps_c,
                                                         const double* __restrict__ intr_c,
                                                         const double* __restrict__ X,
                                                         double* __restrict__ Xc, double radius) {
    constexpr int IW = kIW<CM>;
    __shared__ CamPre scp[kCamSlots], scc[kCamSlots];
    __shared__ double csy[kCamSlots][6];        // camera scaleF * yF (0 for a constant image)
    __shared__ double isy[kIntrSlots][3 * IW];  // intrinsics | candidate | scaleF * yF
    const int c = blockIdx.x, tid = threadIdx.x;
    const double inv_radius = 1.0 / radius;   // as schur_kernel
    const ChunkDesc& cd = P.chunks[c];
    {
        constexpr int kCpW = sizeof(CamPre) / 8;
        for (int e = tid; e < cd.n_cams * kCpW; e += blockDim.x) {
            const int t = e / kCpW, w = e - t * kCpW;
            reinterpret_cast<double*>(&scp[t])[w] = reinterpret_cast<const double*>(&cps[cd.cam_img[t]])[w];
            reinterpret_cast<double*>(&scc[t])[w] = reinterpret_cast<const double*>(&cps_c[cd.cam_img[t]])[w];
        }
        for (int e = tid; e < cd.n_cams * 6; e += blockDim.x) {
            const int t = e / 6, k = e - 6 * t, col = cd.cam_col[t];
            csy[t][k] = col >= 0 ? P.scaleF[col + k] * P.yF[col + k] : 0.0;
        }

        if (tid < IW * cd.n_intr) {
            const int t = tid / IW, k = tid - IW * t, col = cd.intr_col[t];
            isy[t][k] = intr[IW * cd.intr_id[t] + k];
            isy[t][IW + k] = intr_c[IW * cd.intr_id[t] + k];
            isy[t][2 * IW + k] = P.scaleF[col + k] * P.yF[col + k];
        }
    }
    __syncthreads();
    const int p = cd.pt_begin + tid / SPLIT, sub = tid % SPLIT;
    double acc[3] = {0.0, 0.0, 0.0};  // model acc, candidate cost, step norm^2
    double bad = 0.0, cbad = 0.0;     // non-finite step / non-finite candidate residual
    if (p < cd.pt_end) {
        const double Xp[3] = {X[3 * (size_t)p], X[3 * (size_t)p + 1], X[3 * (size_t)p + 2]};
        const double sE[3] = {P.scaleE[3 * (size_t)p], P.scaleE[3 * (size_t)p + 1], P.scaleE[3 * (size_t)p + 2]};
        // One linearisation per observation at x gathers everything the step
        // needs: with j = J_E rows scaled by sE and q = J_F y_F (this row),
        //   V = sum j j',  b = sum j (f - q) = bf - bq,
        // and the model change sum m (f + m/2), m = -(q + j y_E), expands to
        //   -(sum q f + y_E . bf) + (sum q^2 + 2 y_E . bq + y_E' V y_E) / 2.
        double V[6] = {0, 0, 0, 0, 0, 0}, bf[3] = {0, 0, 0}, bq[3] = {0, 0, 0};
        double sqf = 0.0, sqq = 0.0;
        const int o0 = P.pt_off[p] + sub, o1 = P.pt_off[p + 1];
        // the next observation's (slot, uv) is loaded while this one is linearised
        int nslot = o0 < o1 ? P.obs_slot[o0] : 0;
        double2 nuv = o0 < o1 ? reinterpret_cast<const double2*>(P.obs_uv)[o0] : double2{0.0, 0.0};
        for (int o = o0; o < o1; o += SPLIT) {
            const int slot = nslot, cs = slot & 255, is = (slot >> 8) & 255;
            const double2 uv = nuv;
            if (o + SPLIT < o1) {
                nslot = P.obs_slot[o + SPLIT];
                nuv = reinterpret_cast<const double2*>(P.obs_uv)[o + SPLIT];
            }
            LinT<CM> L;
            linearize<CM, true, true, true>(scp[cs], &isy[is][0], Xp, uv.x, uv.y, P.huber_a, L);
            // (a ChunkDesc read: an LDS copy of the flag measured 8 % slower,
            // 94.8 -> 102.5 us at C4, profiles/r03/q_final/step_ab.txt)
            const bool cam = crow_valid(cd, cs);
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                double q = 0.0;  // (J_F y_F) for this row
                if (cam)
#pragma unroll
                    for (int a = 0; a < 6; ++a) q += L.Jc[r][a] * csy[cs][a];
#pragma unroll
                for (int a = 0; a < IW; ++a) q += L.Ji[r][a] * isy[is][2 * IW + a];
                const double j0 = L.Jx[r][0] * sE[0], j1 = L.Jx[r][1] * sE[1], j2 = L.Jx[r][2] * sE[2];
                const double fr = L.f[r];
                V[0] += j0 * j0; V[1] += j1 * j0; V[2] += j1 * j1;
                V[3] += j2 * j0; V[4] += j2 * j1; V[5] += j2 * j2;
                bf[0] += j0 * fr; bf[1] += j1 * fr; bf[2] += j2 * fr;
                bq[0] += j0 * q; bq[1] += j1 * q; bq[2] += j2 * q;
                sqf += q * fr;
                sqq += q * q;
            }
        }
        if constexpr (SPLIT > 1) {
            // the group's partial sums (xor butterfly: the same value in every lane)
#pragma unroll
            for (int m = 1; m < SPLIT; m <<= 1) {
#pragma unroll
                for (int k = 0; k < 6; ++k) V[k] += __shfl_xor(V[k], m);
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    bf[k] += __shfl_xor(bf[k], m);
                    bq[k] += __shfl_xor(bq[k], m);
                }
                sqf += __shfl_xor(sqf, m);
                sqq += __shfl_xor(sqq, m);
            }
        }
        const double V0[6] = {V[0], V[1], V[2], V[3], V[4], V[5]};
        const double b[3] = {bf[0] - bq[0], bf[1] - bq[1], bf[2] - bq[2]};
        const int di[3] = {0, 2, 5};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            V[di[a]] += point_d2(P, V[di[a]], inv_radius);
        }
        // y_E = (V + D^2)^-1 (g_E - W' y_F) via Cholesky
        const double l00 = sqrt(V[0]), l10 = V[1] / l00, l20 = V[3] / l00;
        const double l11 = sqrt(V[2] - l10 * l10), l21 = (V[4] - l20 * l10) / l11;
        const double l22 = sqrt(V[5] - l20 * l20 - l21 * l21);
        const double z0 = b[0] / l00, z1 = (b[1] - l10 * z0) / l11, z2 = (b[2] - l20 * z0 - l21 * z1) / l22;
        const double y2 = z2 / l22, y1 = (z1 - l21 * y2) / l11, y0 = (z0 - l10 * y1 - l20 * y2) / l00;
        const double yE[3] = {y0, y1, y2};
        double xc[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            xc[a] = Xp[a] + (-yE[a]) * sE[a];
            const double d = Xp[a] - xc[a];
            acc[2] += d * d;
            if (sub == 0) Xc[3 * (size_t)p + a] = xc[a];
            if (!isfinite(xc[a])) bad = 1.0;
        }
        {
            const double ybf = yE[0] * bf[0] + yE[1] * bf[1] + yE[2] * bf[2];
            const double ybq = yE[0] * bq[0] + yE[1] * bq[1] + yE[2] * bq[2];
            const double Vy0 = V0[0] * yE[0] + V0[1] * yE[1] + V0[3] * yE[2];
            const double Vy1 = V0[1] * yE[0] + V0[2] * yE[1] + V0[4] * yE[2];
            const double Vy2 = V0[3] * yE[0] + V0[4] * yE[1] + V0[5] * yE[2];
            const double yVy = yE[0] * Vy0 + yE[1] * Vy1 + yE[2] * Vy2;
            acc[0] = -(sqf + ybf) + 0.5 * (sqq + 2.0 * ybq + yVy);
        }
        if (sub != 0) acc[0] = acc[2] = 0.0;   // one lane of the group carries the point's terms
        // candidate residuals at (x_c, candidate cameras / intrinsics)
        nslot = o0 < o1 ? P.obs_slot[o0] : 0;
        nuv = o0 < o1 ? reinterpret_cast<const double2*>(P.obs_uv)[o0] : double2{0.0, 0.0};
        for (int o = o0; o < o1; o += SPLIT) {
            const int slot = nslot, cs = slot & 255, is = (slot >> 8) & 255;
            const double2 uv = nuv;
            if (o + SPLIT < o1) {
                nslot = P.obs_slot[o + SPLIT];
                nuv = reinterpret_cast<const double2*>(P.obs_uv)[o + SPLIT];
            }
            LinT<CM> C;
            linearize<CM, false, false, false>(scc[cs], &isy[is][IW], xc, uv.x, uv.y, P.huber_a, C);
            acc[1] += C.half_rho;
            if (!C.ok) cbad = 1.0;
        }
        if (!isfinite(acc[0])) bad = 1.0;
    }
    wave_sum(acc);
    bad = wave_max(bad);
    cbad = wave_max(cbad);
    __shared__ double red[kStepThreads / 64][kPartT];
    const int wave = tid >> 6, lane = tid & 63, nw = blockDim.x >> 6;
    if (lane == 0) {
        red[wave][0] = acc[0]; red[wave][1] = acc[1]; red[wave][2] = acc[2];
        red[wave][3] = bad; red[wave][4] = cbad;
    }
    __syncthreads();
    if (tid < kPartT) {
        double v = red[0][tid];
        for (int w = 1; w < nw; ++w) v = tid < 3 ? v + red[w][tid] : fmax(v, red[w][tid]);
        P.part_t[kPartT * (size_t)c + tid] = v;
    }
}

// ---------------------------------------------------------------------------
// General points (ba_plan.h): one wavefront per point -- any number of
// observations (rounds of 64), repeated views of one image, any number of
// intrinsics blocks.  The point is eliminated as in schur_kernel (V + D^2, its
// Cholesky L, w = L^-1 g_E, M = Jx L^-T per observation) and its eliminated
// rows Z_b = sum over the observations of block b of J_b' M (camera 6 x 3,
// intrinsics 4 x 3) plus w go to the Z buffer; preduce_kernel forms the RCS
// contributions -Z_a Z_b' and -Z_a w.  The point's Z is accumulated in LDS
// (dynamic: 64 x 19 staging doubles + the largest point's Z) in a fixed order:
// a camera block sums its adjacent run of observations (the planner sorts a
// general point's observations by image), an intrinsics block one masked
// wave sum per 64-observation round, rounds in order.
// ---------------------------------------------------------------------------

constexpr int kZStage = 19;   // doubles per staged observation row (18 used, odd stride)

template <int CM, bool SE>
__global__ __launch_bounds__(64) void zpoint_kernel(DevProblem P, const CamPre* __restrict__ cps,
                                                    const double* __restrict__ intr, const double* __restrict__ X,
                                                    double radius) {
    extern __shared__ __attribute__((aligned(16))) double zlds[];
    double* zc = zlds;                       // [64][kZStage] camera rows J_c' M of this round
    double* Zl = zlds + 64 * kZStage;        // the point's Z (blocks), accumulated
    __shared__ int cbl[64];
    const int lane = threadIdx.x, g = P.zlong[blockIdx.x];
    const int k = P.n_cpt + g;
    const int o0 = P.pt_off[k], o1 = P.pt_off[k + 1];
    const int b0 = P.gblk_off[g];
    const int zn = (int)(P.gz_off[g + 1] - P.gz_off[g]) - 3;
    const double Xp[3] = {X[3 * (size_t)k], X[3 * (size_t)k + 1], X[3 * (size_t)k + 2]};
    double sE[3];
    // observation o at x: loss-corrected Jacobians, unscaled
    constexpr int IW = kIW<CM>;
    auto lin = [&](int o, LinT<CM>& L) {
        const int img = P.obs_img[o];
        const double2 uv = reinterpret_cast<const double2*>(P.obs_uv)[o];
        linearize<CM, true, true, true>(cps[img], intr + IW * (size_t)P.img_intr[img], Xp, uv.x, uv.y, P.huber_a, L);
    };
    if constexpr (SE) {
        // the solve's first pass: Ceres' Jacobi point scales from the column
        // norms of the unscaled point Jacobian
        double cn[3] = {0.0, 0.0, 0.0};
        for (int o = o0 + lane; o < o1; o += 64) {
            LinT<CM> L;
            lin(o, L);
#pragma unroll
            for (int a = 0; a < 3; ++a) cn[a] += L.Jx[0][a] * L.Jx[0][a] + L.Jx[1][a] * L.Jx[1][a];
        }
        wave_sum(cn);
#pragma unroll
        for (int a = 0; a < 3; ++a) sE[a] = 1.0 / (1.0 + sqrt(cn[a]));
        if (lane < 3) P.scaleE[3 * (size_t)k + lane] = sE[lane];
    } else {
#pragma unroll
        for (int a = 0; a < 3; ++a) sE[a] = P.scaleE[3 * (size_t)k + a];
    }
    // V = Jx' Jx, g_E = Jx' f over the point (scaled), summed by the wave
    double v9[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};   // V00 V10 V11 V20 V21 V22 | b0 b1 b2
    for (int o = o0 + lane; o < o1; o += 64) {
        LinT<CM> L;
        lin(o, L);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const double j0 = L.Jx[r][0] * sE[0], j1 = L.Jx[r][1] * sE[1], j2 = L.Jx[r][2] * sE[2], fr = L.f[r];
            v9[0] += j0 * j0; v9[1] += j1 * j0; v9[2] += j1 * j1;
            v9[3] += j2 * j0; v9[4] += j2 * j1; v9[5] += j2 * j2;
            v9[6] += j0 * fr; v9[7] += j1 * fr; v9[8] += j2 * fr;
        }
    }
    wave_sum(v9);
    double V[6] = {v9[0], v9[1], v9[2], v9[3], v9[4], v9[5]};
    const double b[3] = {v9[6], v9[7], v9[8]};
    if (lane == 0) {   // gradient / norm bookkeeping at x
        double xn2 = 0.0, gmx = 0.0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const double gg = b[a] * rcp_nr(sE[a]);
            xn2 += Xp[a] * Xp[a];
            gmx = fmax(gmx, fabs(Xp[a] - (Xp[a] - gg)));
        }
        P.part_s[2 * (size_t)(P.n_chunk + g)] = xn2;
        P.part_s[2 * (size_t)(P.n_chunk + g) + 1] = gmx;
    }
    const double inv_radius = 1.0 / radius;
    const int di[3] = {0, 2, 5};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        V[di[a]] += point_d2(P, V[di[a]], inv_radius);
    }
    const double i00 = rsqrt_nr(V[0]);
    const double l10 = V[1] * i00, l20 = V[3] * i00;
    const double i11 = rsqrt_nr(V[2] - l10 * l10);
    const double l21 = (V[4] - l20 * l10) * i11;
    const double i22 = rsqrt_nr(V[5] - l20 * l20 - l21 * l21);
    const double i10 = -l10 * i00 * i11, i21 = -l21 * i11 * i22;
    const double i20 = -(l20 * i00 + l21 * i10) * i22;
    for (int e = lane; e < zn; e += 64) Zl[e] = 0.0;
    int prev_cb = -1;   // camera block of the previous round's last observation
    for (int base = o0; base < o1; base += 64) {
        const int o = base + lane;
        const bool act = o < o1;
        int cb = 0xffff, ib = -1;
        double zi[3 * IW];
#pragma unroll
        for (int e = 0; e < 3 * IW; ++e) zi[e] = 0.0;
        if (act) {
            LinT<CM> L;
            lin(o, L);
            const int img = P.obs_img[o];
            const int slot = P.obs_slot[o];
            cb = slot & 0xffff;
            ib = slot >> 16;
            double M[2][3];
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const double j0 = L.Jx[r][0] * sE[0], j1 = L.Jx[r][1] * sE[1], j2 = L.Jx[r][2] * sE[2];
                M[r][0] = j0 * i00;
                M[r][1] = j0 * i10 + j1 * i11;
                M[r][2] = j0 * i20 + j1 * i21 + j2 * i22;
            }
            const int colc = P.img_colc[img], coli = P.img_coli[img];
            if (cb != 0xffff) {
#pragma unroll
                for (int r = 0; r < 6; ++r) {
                    const double s = P.scaleF[colc + r];
#pragma unroll
                    for (int a = 0; a < 3; ++a)
                        zc[lane * kZStage + 3 * r + a] = (L.Jc[0][r] * s) * M[0][a] + (L.Jc[1][r] * s) * M[1][a];
                }
            }
            const int ni = CM == SFM_CAM_SNAVELY ? 3 : IW;
#pragma unroll
            for (int r = 0; r < IW; ++r) {
                if (r >= ni) continue;
                const double s = P.scaleF[coli + r];
#pragma unroll
                for (int a = 0; a < 3; ++a) zi[3 * r + a] = (L.Ji[0][r] * s) * M[0][a] + (L.Ji[1][r] * s) * M[1][a];
            }
        }
        cbl[lane] = act ? cb : -2;
        wsync();
        // camera blocks: the first observation of each run sums the run in order
        const bool head = act && cb != 0xffff && (lane == 0 || cbl[lane - 1] != cb);
        if (head) {
            double acc[18];
#pragma unroll
            for (int e = 0; e < 18; ++e) acc[e] = zc[lane * kZStage + e];
            for (int q = lane + 1; q < 64 && cbl[q] == cb; ++q)
#pragma unroll
                for (int e = 0; e < 18; ++e) acc[e] += zc[q * kZStage + e];
            double* dst = Zl + P.gblk_z[b0 + cb];
            const bool cont = lane == 0 && cb == prev_cb;   // run continued from the previous round
#pragma unroll
            for (int e = 0; e < 18; ++e) dst[e] = cont ? dst[e] + acc[e] : acc[e];
        }
        prev_cb = cbl[63] >= 0 ? cbl[63] : -1;
        // intrinsics blocks: one masked wave sum per distinct block of the round
        unsigned long long pend = __ballot(act);
        while (pend) {
            const int src = __builtin_ctzll(pend);
            const int j = __shfl(ib, src);
            const bool mine = act && ib == j;
            double v[3 * IW];
#pragma unroll
            for (int e = 0; e < 3 * IW; ++e) v[e] = mine ? zi[e] : 0.0;
            wave_sum(v);
            const int nz = 3 * (CM == SFM_CAM_SNAVELY ? 3 : IW);
            double mine_v = 0.0;   // v[lane] without a dynamically indexed register array
#pragma unroll
            for (int e = 0; e < 3 * IW; ++e) mine_v = lane == e ? v[e] : mine_v;
            if (lane < nz) Zl[P.gblk_z[b0 + j] + lane] += mine_v;
            pend &= ~__ballot(mine);
        }
        wsync();
    }
    double* Zg = P.Z + P.gz_off[g];
    for (int e = lane; e < zn; e += 64) Zg[e] = Zl[e];
    if (lane < 3) {
        const double w3[3] = {i00 * b[0], i10 * b[0] + i11 * b[1], i20 * b[0] + i21 * b[1] + i22 * b[2]};
        Zg[zn + lane] = lane == 0 ? w3[0] : lane == 1 ? w3[1] : w3[2];
    }
}

// Short general points (<= kZShortObs observations), a batch of consecutive
// points per wave, one lane per observation (zpoint_kernel spent a wave on
// each point, 10 of 64 lanes busy at random-k visibility, and linearised every
// observation twice).  Each observation is linearised once; every per-point
// sum (column norms, V | g_E, a camera block's run, an intrinsics block) is
// taken by the first lane of its group over the group's LDS rows in
// observation order, so the result is fixed.
constexpr int kZRow = 19;   // LDS row stride (doubles) of a lane's staged values
template <int CM, bool SE>
__global__ __launch_bounds__(64) void zbatch_kernel(DevProblem P, const CamPre* __restrict__ cps,
                                                    const double* __restrict__ intr, const double* __restrict__ X,
                                                    double radius) {
    constexpr int IW = kIW<CM>;
    constexpr int NI = CM == SFM_CAM_SNAVELY ? 3 : IW;   // intrinsics parameters with a column
    // camera rows J_c' M (18), then (round 6: one array, not two -- 2 -> 3
    // workgroups per SIMD) the intrinsics rows J_i' M (3 NI); before them
    // V | g_E (9), column norms (3)
    __shared__ double rc[64][kZRow];
    __shared__ double pv[kZBatchPts][12]; // per point: V (6) | g_E (3) | sE (3)
    __shared__ int poff[kZBatchPts + 1], okey[64], oib[64];
    const int lane = threadIdx.x;
    const int g0 = P.zbatch[2 * blockIdx.x], g1 = P.zbatch[2 * blockIdx.x + 1], np = g1 - g0;
    const int oA = P.pt_off[P.n_cpt + g0];
    if (lane <= np) poff[lane] = P.pt_off[P.n_cpt + g0 + lane] - oA;
    wsync();
    const int nobs = poff[np];
    const bool act = lane < nobs;
    int pl = 0;   // this lane's point within the batch
    for (int j = 1; j < np; ++j) pl += poff[j] <= lane ? 1 : 0;
    const int g = g0 + pl, k = P.n_cpt + g, o = oA + lane;
    const bool head = act && lane == poff[pl];   // the point's first observation
    double Xp[3] = {0.0, 0.0, 0.0};
    LinT<CM> L{};
    int img = 0, cb = 0xffff, ib = 0;
    if (act) {
#pragma unroll
        for (int a = 0; a < 3; ++a) Xp[a] = X[3 * (size_t)k + a];
        img = P.obs_img[o];
        const int slot = P.obs_slot[o];
        cb = slot & 0xffff;
        ib = slot >> 16;
        const double2 uv = reinterpret_cast<const double2*>(P.obs_uv)[o];
        linearize<CM, true, true, true>(cps[img], intr + IW * (size_t)P.img_intr[img], Xp, uv.x, uv.y, P.huber_a, L);
    }
    // per-point sums of n values staged in rc by every lane: the head lane adds
    // its point's rows in order into pv[pl][at..at+n)
    auto point_sum = [&](int n, int at) {
        wsync();
        if (head) {
            for (int e = 0; e < n; ++e) {
                double acc = rc[lane][e];
                for (int q = lane + 1; q < poff[pl + 1]; ++q) acc += rc[q][e];
                pv[pl][at + e] = acc;
            }
        }
        wsync();
    };
    double sE[3];
    if constexpr (SE) {
        // the solve's first pass: Ceres' Jacobi point scales from the column
        // norms of the unscaled point Jacobian
        if (act)
#pragma unroll
            for (int a = 0; a < 3; ++a) rc[lane][a] = L.Jx[0][a] * L.Jx[0][a] + L.Jx[1][a] * L.Jx[1][a];
        point_sum(3, 9);
        if (head)
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const double se = 1.0 / (1.0 + sqrt(pv[pl][9 + a]));
                pv[pl][9 + a] = se;
                P.scaleE[3 * (size_t)k + a] = se;
            }
        wsync();
#pragma unroll
        for (int a = 0; a < 3; ++a) sE[a] = pv[pl][9 + a];
    } else {
#pragma unroll
        for (int a = 0; a < 3; ++a) sE[a] = act ? P.scaleE[3 * (size_t)k + a] : 1.0;
    }
    // V = Jx' Jx, g_E = Jx' f per point (scaled)
    double j[2][3];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int a = 0; a < 3; ++a) j[r][a] = L.Jx[r][a] * sE[a];
    if (act) {
        double v9[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const double fr = L.f[r];
            v9[0] += j[r][0] * j[r][0]; v9[1] += j[r][1] * j[r][0]; v9[2] += j[r][1] * j[r][1];
            v9[3] += j[r][2] * j[r][0]; v9[4] += j[r][2] * j[r][1]; v9[5] += j[r][2] * j[r][2];
            v9[6] += j[r][0] * fr; v9[7] += j[r][1] * fr; v9[8] += j[r][2] * fr;
        }
#pragma unroll
        for (int e = 0; e < 9; ++e) rc[lane][e] = v9[e];
    }
    point_sum(9, 0);
    double V[6], b[3];
#pragma unroll
    for (int e = 0; e < 6; ++e) V[e] = pv[pl][e];
#pragma unroll
    for (int e = 0; e < 3; ++e) b[e] = pv[pl][6 + e];
    if (head) {   // gradient / norm bookkeeping at x
        double xn2 = 0.0, gmx = 0.0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const double gg = b[a] * rcp_nr(sE[a]);
            xn2 += Xp[a] * Xp[a];
            gmx = fmax(gmx, fabs(Xp[a] - (Xp[a] - gg)));
        }
        P.part_s[2 * (size_t)(P.n_chunk + g)] = xn2;
        P.part_s[2 * (size_t)(P.n_chunk + g) + 1] = gmx;
    }
    const double inv_radius = 1.0 / radius;
    const int di[3] = {0, 2, 5};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        V[di[a]] += point_d2(P, V[di[a]], inv_radius);
    }
    const double i00 = rsqrt_nr(V[0]);
    const double l10 = V[1] * i00, l20 = V[3] * i00;
    const double i11 = rsqrt_nr(V[2] - l10 * l10);
    const double l21 = (V[4] - l20 * l10) * i11;
    const double i22 = rsqrt_nr(V[5] - l20 * l20 - l21 * l21);
    const double i10 = -l10 * i00 * i11, i21 = -l21 * i11 * i22;
    const double i20 = -(l20 * i00 + l21 * i10) * i22;
    double M[2][3];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        M[r][0] = j[r][0] * i00;
        M[r][1] = j[r][0] * i10 + j[r][1] * i11;
        M[r][2] = j[r][0] * i20 + j[r][1] * i21 + j[r][2] * i22;
    }
    if (act) {
        if (cb != 0xffff) {
            const int colc = P.img_colc[img];
#pragma unroll
            for (int r = 0; r < 6; ++r) {
                const double sc = P.scaleF[colc + r];
#pragma unroll
                for (int a = 0; a < 3; ++a) rc[lane][3 * r + a] = (L.Jc[0][r] * sc) * M[0][a] + (L.Jc[1][r] * sc) * M[1][a];
            }
        }
    }
    okey[lane] = act ? (pl << 17 | cb) : -1;
    oib[lane] = ib;
    wsync();
    double* Zp = P.Z + P.gz_off[g];
    const int b0 = P.gblk_off[g], pend = poff[pl + 1];
    if (act) {
        // camera block: the first lane of a run of one (point, camera block)
        // adds the run in order (the planner sorts a point's views by image)
        if (cb != 0xffff && (lane == poff[pl] || okey[lane - 1] != okey[lane])) {
            double acc[18];
#pragma unroll
            for (int e = 0; e < 18; ++e) acc[e] = rc[lane][e];
            for (int q = lane + 1; q < pend && okey[q] == okey[lane]; ++q)
#pragma unroll
                for (int e = 0; e < 18; ++e) acc[e] += rc[q][e];
            double* dst = Zp + P.gblk_z[b0 + cb];
#pragma unroll
            for (int e = 0; e < 18; ++e) dst[e] = acc[e];
        }
    }
    wsync();   // (the camera rows are read; the intrinsics rows take their place)
    if (act) {
        const int coli = P.img_coli[img];
#pragma unroll
        for (int r = 0; r < NI; ++r) {
            const double sc = P.scaleF[coli + r];
#pragma unroll
            for (int a = 0; a < 3; ++a) rc[lane][3 * r + a] = (L.Ji[0][r] * sc) * M[0][a] + (L.Ji[1][r] * sc) * M[1][a];
        }
    }
    wsync();
    if (act) {
        // intrinsics block: the point's first lane with that block adds all of
        // the point's lanes with it, in order
        bool first = true;
        for (int q = poff[pl]; q < lane; ++q) first = first && oib[q] != ib;
        if (first) {
            double acc[3 * NI];
#pragma unroll
            for (int e = 0; e < 3 * NI; ++e) acc[e] = rc[lane][e];
            for (int q = lane + 1; q < pend; ++q)
                if (oib[q] == ib)
#pragma unroll
                    for (int e = 0; e < 3 * NI; ++e) acc[e] += rc[q][e];
            double* dst = Zp + P.gblk_z[b0 + ib];
#pragma unroll
            for (int e = 0; e < 3 * IW; ++e) dst[e] = e < 3 * NI ? acc[e < 3 * NI ? e : 0] : 0.0;   // SNAVELY: row 3 is 0
        }
        if (head) {   // w = L^-1 g_E after the point's blocks
            const int zn = (int)(P.gz_off[g + 1] - P.gz_off[g]) - 3;
            Zp[zn] = i00 * b[0];
            Zp[zn + 1] = i10 * b[0] + i11 * b[1];
            Zp[zn + 2] = i20 * b[0] + i21 * b[1] + i22 * b[2];
        }
    }
}

// Product terms of the general points: target element (r, c) -= sum over the
// target's terms (in order) of Z_a[r] . Z_b[c] (3-vectors).  One wave per
// target, one lane per element; runs after reduce_kernel has written the sum
// terms.
// Lists longer than this (the intrinsics arrow and corner collect one term
// per general point) go through preduce_seg_kernel + preduce_long_kernel.
constexpr int kLongPTerms = 64;

// sum over the product terms q = qa + g, qa + g + G, ... < qb of
// Z_a[3r..3r+2] . Z_b[3cc..3cc+2] (ascending, one term after another, as a
// plain per-lane loop would).  The Z blocks are staged through LDS kPtB terms
// at a time: the wave loads each term's two blocks once, coalesced (the rows
// are contiguous 3-vectors), instead of every lane gathering its own six
// doubles per term (36 lanes x 6 scattered 8-byte loads per term made the
// reduce address-bound).  Round 6: in 16-byte pieces -- a term's two blocks
// are ceil(3 ra / 2) + ceil(3 rb / 2) pieces (18 for 6 x 6), the batch's 288
// pieces five wave loads instead of sixteen 8-byte ones -- each piece's two
// doubles put in their padded LDS places.  Rows are padded to 4 doubles in
// LDS (two 16-byte reads per 3-vector).  ra / rb: rows of the a / b block
// (b = w: 1 row).
constexpr int kPtB = 16;   // terms per staged batch of the product-term reduce
constexpr int kPtLds = kPtB * 12 * 4 + 2 * kPtB;   // doubles of LDS per wave (<= 6 + 6 rows per term, the terms)
constexpr int kPtRounds = (kPtB * 18 + 63) / 64;   // a lane's 16-byte pieces per batch
typedef double d2u __attribute__((ext_vector_type(2), aligned(8)));   // (Z blocks are 8-byte aligned)
// ch > 0 (a block target with an even number of columns, round 6): the lane
// also sums element (r, cc + ch) into s1 -- one read of Z_a's row r for two
// elements, and half the lanes per element, so three lane groups share a
// 6 x 6 target's terms instead of one (36 of 64 lanes)
__device__ __forceinline__ double pterm_sum(const DevProblem& P, int qa, int qb, int G, int g, int r, int cc,
                                            int ra, int rb, double* lds, int ch, double& s1) {
    const double* Z = P.Z;
    const int lane = threadIdx.x & 63;
    const int la = 3 * ra, lb = 3 * rb;                          // doubles per a / b block
    const int na2 = (la + 1) >> 1, n2 = na2 + ((lb + 1) >> 1);   // 16-byte pieces per term
    double* La = lds;                          // [kPtB][ra][4]
    double* Lb = lds + kPtB * ra * 4;          // [kPtB][rb][4]
    PTerm* Lt = reinterpret_cast<PTerm*>(lds + kPtB * 12 * 4);   // [kPtB] the batch's terms
    // this lane's pieces (the same in every batch): piece f = lane + 64 q is
    // term f / n2's piece o = f % n2, doubles 2o, 2o + 1 of its a block (o <
    // na2) or of its b block; an odd block's last piece carries one double
    // (its second is read and dropped: Z is allocated two doubles longer)
    int pt[kPtRounds], pe[kPtRounds], d0[kPtRounds], d1[kPtRounds];
#pragma unroll
    for (int q = 0; q < kPtRounds; ++q) {
        const int f = lane + 64 * q, t = f / n2, o = f - t * n2;
        const bool sb = o >= na2;
        const int e = sb ? 2 * (o - na2) : 2 * o, len = sb ? lb : la;
        const int rows = sb ? rb : ra, base = (sb ? kPtB * ra * 4 : 0) + t * rows * 4;
        pt[q] = t < kPtB ? t : kPtB;
        pe[q] = e | (sb ? 256 : 0);
        d0[q] = base + (e / 3) * 4 + e % 3;
        d1[q] = e + 1 < len ? base + ((e + 1) / 3) * 4 + (e + 1) % 3 : -1;
    }
    double s = 0.0;
    s1 = 0.0;
    // software pipeline: batch b + 1's pieces are loaded into registers while
    // batch b is multiplied from LDS, and batch b + 2's term offsets with them
    // (two scalars, not a PTerm: the struct was promoted to LDS, and its
    // store there waited for the load it was meant to prefetch)
    const int2* pt2 = reinterpret_cast<const int2*>(P.pterms);
    int2 nxt = make_int2(0, 0);
    auto load_offs = [&](int q0) {   // batch q0's term offsets -> nxt
        if (lane < min(kPtB, qb - q0)) nxt = pt2[q0 + lane];
    };
    d2u v[kPtRounds];
    auto load_pieces = [&](int nb) {   // the staged batch's (Lt) pieces -> v
        // every piece's load in flight at once (unconditional: pieces past
        // the batch read term 0's first piece)
#pragma unroll
        for (int q = 0; q < kPtRounds; ++q) {
            const bool live = pt[q] < nb;
            const PTerm tm = Lt[live ? pt[q] : 0];
            const int32_t off = live ? ((pe[q] & 256) ? tm.zb : tm.za) + (pe[q] & 255) : tm.za;
            v[q] = *reinterpret_cast<const d2u*>(Z + off);
        }
    };
    if (qa >= qb) return s;
    load_offs(qa);
    int nb = min(kPtB, qb - qa);
    if (lane < nb) Lt[lane] = PTerm{nxt.x, nxt.y};
    load_offs(qa + kPtB);
    wsync();
    load_pieces(nb);
    for (int q0 = qa; q0 < qb; q0 += kPtB) {
        wsync();   // (the previous batch's reads of La / Lb and Lt are done)
#pragma unroll
        for (int q = 0; q < kPtRounds; ++q)
            if (pt[q] < nb) {
                lds[d0[q]] = v[q].x;
                if (d1[q] >= 0) lds[d1[q]] = v[q].y;
            }
        // the next batch: its offsets to Lt, its pieces in flight
        const int q1 = q0 + kPtB, nb1 = min(kPtB, qb - q1);
        if (nb1 > 0 && lane < nb1) Lt[lane] = PTerm{nxt.x, nxt.y};
        if (nb1 > 0) load_offs(q1 + kPtB);
        wsync();
        if (nb1 > 0) load_pieces(nb1);
        if (g >= 0) {
            // this group's terms in the batch: j = g - (q0 - qa) mod G, + G, ...
            int j = (g - (q0 - qa) % G + G) % G;
            for (; j < nb; j += G) {
                const double2 a01 = *reinterpret_cast<const double2*>(La + (j * ra + r) * 4);
                const double a2 = La[(j * ra + r) * 4 + 2];
                const double2 b01 = *reinterpret_cast<const double2*>(Lb + (j * rb + cc) * 4);
                const double b2 = Lb[(j * rb + cc) * 4 + 2];
                s += a01.x * b01.x + a01.y * b01.y + a2 * b2;
                if (ch) {
                    const double2 c01 = *reinterpret_cast<const double2*>(Lb + (j * rb + cc + ch) * 4);
                    const double c2 = Lb[(j * rb + cc + ch) * 4 + 2];
                    s1 += a01.x * c01.x + a01.y * c01.y + a2 * c2;
                }
            }
        }
        nb = nb1;
    }
    wsync();
    return s;
}

// A product-term target's lane layout: E2 lane slots of one element (r, cc)
// -- or two, (r, cc) and (r, cc + ch), when the target has an even number of
// columns -- in G = 64 / E2 lane groups; slot e2 = r * (ch ? ch : cols) + cc.
struct PLanes {
    int E2, G, g, r, cc, ch;
    __device__ __forceinline__ PLanes(const ReduceTarget& T, int lane) {
        const bool vec = T.cols == 1;
        ch = (!vec && (T.cols & 1) == 0) ? T.cols / 2 : 0;
        const int w = ch ? ch : T.cols;
        E2 = T.rows * w;
        G = 64 / E2;
        g = lane / E2;
        const int e2 = lane - g * E2;
        r = e2 / w;
        cc = e2 % w;
        if (g >= G) g = -1;
    }
    // element e (= r * cols + c) of the target: its slot and which sum
    __device__ __forceinline__ int slot(const ReduceTarget& T, int e, bool& second) const {
        const int rr = e / T.cols, c = e % T.cols;
        second = ch && c >= ch;
        return rr * (ch ? ch : T.cols) + (second ? c - ch : c);
    }
};

// One wave per target: its E = rows x cols elements are computed by
// G = 64 / E lane groups, group g summing terms g, g + G, ... (a 6-vector
// target keeps 60 lanes busy, a 6x6 block 36); the group partials are then
// added in group order (fixed, so deterministic).
__global__ __launch_bounds__(256) void preduce_kernel(DevProblem P) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + wave;
    __shared__ double part[4][64];
    ReduceTarget T{};
    bool act = t < P.n_targets;
    if (act) {
        T = P.targets[t];
        act = T.p_end > T.p_begin && T.p_end - T.p_begin <= kLongPTerms;
    }
    if (!act) return;   // whole waves only: the exchange below is wave-local
    __shared__ __attribute__((aligned(16))) double stage[4][kPtLds];
    __shared__ double part1[4][64];
    const PLanes pl(T, lane);
    const int E = T.rows * T.cols;
    const bool vec = T.cols == 1;
    double s1;
    const double s = pterm_sum(P, T.p_begin, T.p_end, pl.G, pl.g, pl.r, pl.cc, T.rows, vec ? 1 : T.cols, stage[wave],
                               pl.ch, s1);
    part[wave][lane] = s;
    part1[wave][lane] = s1;
    wsync();
    if (lane < E) {
        bool second;
        const int e2 = pl.slot(T, lane, second);
        const double* src = second ? part1[wave] : part[wave];
        double tot = 0.0;
        for (int k = 0; k < pl.G; ++k) tot += src[k * pl.E2 + e2];
        const int r = lane / T.cols, cc = lane % T.cols;
        target_base(P, T.dst_kind)[T.dst + (vec ? r : (int64_t)r * T.ld + cc)] -= tot;
    }
}

// Long product-term lists, pass 1: one workgroup per kReduceSeg-term segment,
// each wave a quarter of it, laid out as in preduce_kernel (G lane groups of
// E elements); the partials added in (wave, group) order, fixed.
__global__ __launch_bounds__(256) void preduce_seg_kernel(DevProblem P) {
    const int sg = blockIdx.x;
    const int j = P.plseg[2 * sg], k0 = P.plseg[2 * sg + 1];
    const ReduceTarget T = P.targets[P.plong_targets[j]];
    const int E = T.rows * T.cols;
    const bool vec = T.cols == 1;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const PLanes pl(T, lane);
    constexpr int kQ = kReduceSeg / 4;
    const int q0 = k0 + wave * kQ, q1 = min(min(k0 + kReduceSeg, (int)T.p_end), q0 + kQ);
    __shared__ __attribute__((aligned(16))) double stage[4][kPtLds];
    double s1 = 0.0;
    const double s = q0 < q1 ? pterm_sum(P, q0, q1, pl.G, pl.g, pl.r, pl.cc, T.rows, vec ? 1 : T.cols, stage[wave],
                                         pl.ch, s1)
                             : 0.0;
    __shared__ double part[4][64], part1[4][64];
    part[wave][lane] = s;
    part1[wave][lane] = s1;
    __syncthreads();
    if ((int)threadIdx.x < E) {
        const int t = threadIdx.x;
        bool second;
        const int e2 = pl.slot(T, t, second);
        double tot = 0.0;
        for (int w = 0; w < 4; ++w)
            for (int k = 0; k < pl.G; ++k) tot += (second ? part1[w] : part[w])[k * pl.E2 + e2];
        P.plpart[(size_t)sg * 36 + t] = tot;
    }
}

// pass 2: segment partials added in segment order, subtracted from the target
__global__ __launch_bounds__(64) void preduce_long_kernel(DevProblem P) {
    const int j = blockIdx.x;
    const ReduceTarget T = P.targets[P.plong_targets[j]];
    const int E = T.rows * T.cols, e = threadIdx.x;
    if (e >= E) return;
    double t = 0.0;
#pragma unroll 8
    for (int sg = P.plseg_off[j]; sg < P.plseg_off[j + 1]; ++sg) t += P.plpart[(size_t)sg * 36 + e];
    const int r = e / T.cols, cc = e % T.cols;
    target_base(P, T.dst_kind)[T.dst + (T.cols == 1 ? r : (int64_t)r * T.ld + cc)] -= t;
}

// Step for general points: one thread per point, the same arithmetic as
// step_kernel with cameras and column scales read from global memory.
template <int CM>
__global__ __launch_bounds__(kGStepThreads) void step_general_kernel(
    DevProblem P, const CamPre* __restrict__ cps, const double* __restrict__ intr, const CamPre* __restrict__ cps_c,
    const double* __restrict__ intr_c, const double* __restrict__ X, double* __restrict__ Xc, double radius) {
    constexpr int IW = kIW<CM>;
    const int tid = threadIdx.x, g = blockIdx.x * kGStepThreads + tid;
    const double inv_radius = 1.0 / radius;
    double acc[3] = {0.0, 0.0, 0.0};
    double bad = 0.0, cbad = 0.0;
    if (g < P.n_gpt) {
        const int p = P.n_cpt + g;
        const double Xp[3] = {X[3 * (size_t)p], X[3 * (size_t)p + 1], X[3 * (size_t)p + 2]};
        const double sE[3] = {P.scaleE[3 * (size_t)p], P.scaleE[3 * (size_t)p + 1], P.scaleE[3 * (size_t)p + 2]};
        double V[6] = {0, 0, 0, 0, 0, 0}, bf[3] = {0, 0, 0}, bq[3] = {0, 0, 0};
        double sqf = 0.0, sqq = 0.0;
        const int o0 = P.pt_off[p], o1 = P.pt_off[p + 1];
        for (int o = o0; o < o1; ++o) {
            const int img = P.obs_img[o];
            const double2 uv = reinterpret_cast<const double2*>(P.obs_uv)[o];
            const int colc = P.img_colc[img], coli = P.img_coli[img];
            LinT<CM> L;
            linearize<CM, true, true, true>(cps[img], intr + IW * (size_t)P.img_intr[img], Xp, uv.x, uv.y, P.huber_a, L);
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                double q = 0.0;
                if (colc >= 0)
#pragma unroll
                    for (int a = 0; a < 6; ++a) q += L.Jc[r][a] * (P.scaleF[colc + a] * P.yF[colc + a]);
                const int ni = CM == SFM_CAM_SNAVELY ? 3 : IW;
#pragma unroll
                for (int a = 0; a < IW; ++a)
                    if (a < ni) q += L.Ji[r][a] * (P.scaleF[coli + a] * P.yF[coli + a]);
                const double j0 = L.Jx[r][0] * sE[0], j1 = L.Jx[r][1] * sE[1], j2 = L.Jx[r][2] * sE[2];
                const double fr = L.f[r];
                V[0] += j0 * j0; V[1] += j1 * j0; V[2] += j1 * j1;
                V[3] += j2 * j0; V[4] += j2 * j1; V[5] += j2 * j2;
                bf[0] += j0 * fr; bf[1] += j1 * fr; bf[2] += j2 * fr;
                bq[0] += j0 * q; bq[1] += j1 * q; bq[2] += j2 * q;
                sqf += q * fr;
                sqq += q * q;
            }
        }
        const double V0[6] = {V[0], V[1], V[2], V[3], V[4], V[5]};
        const double b[3] = {bf[0] - bq[0], bf[1] - bq[1], bf[2] - bq[2]};
        const int di[3] = {0, 2, 5};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            V[di[a]] += point_d2(P, V[di[a]], inv_radius);
        }
        const double l00 = sqrt(V[0]), l10 = V[1] / l00, l20 = V[3] / l00;
        const double l11 = sqrt(V[2] - l10 * l10), l21 = (V[4] - l20 * l10) / l11;
        const double l22 = sqrt(V[5] - l20 * l20 - l21 * l21);
        const double z0 = b[0] / l00, z1 = (b[1] - l10 * z0) / l11, z2 = (b[2] - l20 * z0 - l21 * z1) / l22;
        const double y2 = z2 / l22, y1 = (z1 - l21 * y2) / l11, y0 = (z0 - l10 * y1 - l20 * y2) / l00;
        const double yE[3] = {y0, y1, y2};
        double xc[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            xc[a] = Xp[a] + (-yE[a]) * sE[a];
            const double d = Xp[a] - xc[a];
            acc[2] += d * d;
            Xc[3 * (size_t)p + a] = xc[a];
            if (!isfinite(xc[a])) bad = 1.0;
        }
        {
            const double ybf = yE[0] * bf[0] + yE[1] * bf[1] + yE[2] * bf[2];
            const double ybq = yE[0] * bq[0] + yE[1] * bq[1] + yE[2] * bq[2];
            const double Vy0 = V0[0] * yE[0] + V0[1] * yE[1] + V0[3] * yE[2];
            const double Vy1 = V0[1] * yE[0] + V0[2] * yE[1] + V0[4] * yE[2];
            const double Vy2 = V0[3] * yE[0] + V0[4] * yE[1] + V0[5] * yE[2];
            const double yVy = yE[0] * Vy0 + yE[1] * Vy1 + yE[2] * Vy2;
            acc[0] = -(sqf + ybf) + 0.5 * (sqq + 2.0 * ybq + yVy);
        }
        for (int o = o0; o < o1; ++o) {
            const int img = P.obs_img[o];
            const double2 uv = reinterpret_cast<const double2*>(P.obs_uv)[o];
            LinT<CM> C;
            linearize<CM, false, false, false>(cps_c[img], intr_c + IW * (size_t)P.img_intr[img], xc, uv.x, uv.y,
                                               P.huber_a, C);
            acc[1] += C.half_rho;
            if (!C.ok) cbad = 1.0;
        }
        if (!isfinite(acc[0])) bad = 1.0;
    }
    wave_sum(acc);
    bad = wave_max(bad);
    cbad = wave_max(cbad);
    constexpr int kW = kGStepThreads / 64;
    __shared__ double red[kW][kPartT];
    const int wave = tid >> 6, lane = tid & 63;
    if (lane == 0) {
        red[wave][0] = acc[0]; red[wave][1] = acc[1]; red[wave][2] = acc[2];
        red[wave][3] = bad; red[wave][4] = cbad;
    }
    __syncthreads();
    if (tid < kPartT) {
        double v = red[0][tid];
        for (int w = 1; w < kW; ++w) v = tid < 3 ? v + red[w][tid] : fmax(v, red[w][tid]);
        P.part_t[kPartT * (size_t)(P.n_chunk + blockIdx.x) + tid] = v;
    }
}

// fixed-order reduction of the per-block partials, in kFinBlocks
// workgroups: workgroup g sums elements g * kFinThreads + t, stepping by
// kFinBlocks * kFinThreads (every thread's loads in flight together), stores
// its 12 partials write-through and takes a ticket; the last to arrive adds
// the partials in workgroup order and publishes (Guideline 16, counter form).
// One 1024-thread workgroup walking every list took 12-13 us at C4 (a chain
// of dependent loads per thread); the sums are now in a different (still
// fixed) order.
// The host's accept decision for this iteration's step (ba_solver.cpp
// run_plan, "this iteration": an invalid step, the parameter and function
// tolerance tests, then the relative decrease), restated on the scalars just
// combined, same operations in the same order -- so the speculative Gram pass
// at the candidate (ba_image_gram with gate) runs exactly when the host will
// accept.  The host still checks the flag against its own decision (and runs
// or redoes the pass on a mismatch), so no result depends on this copy.
__device__ __forceinline__ bool lm_spec_accept(const double* sc, const DevProblem& P) {
    const double model_change = -sc[kScModelAcc];
    const bool finite = sc[kScSolveFail] == 0.0 && sc[kScStepBad] == 0.0 && isfinite(model_change);
    if (!(finite && model_change > 0.0)) return false;
    const double x_cost = sc[kScCost];
    const double cand_cost = sc[kScCandBad] != 0.0 ? DBL_MAX : sc[kScCandCost];
    const double x_norm = sqrt(sc[kScXnorm2E] + sc[kScXnorm2F]);
    const double step_norm = sqrt(sc[kScStepnorm2E] + sc[kScStepnorm2F]);
    if (step_norm <= P.lm_ptol * (x_norm + P.lm_ptol)) return false;
    if (fabs(x_cost - cand_cost) <= P.lm_ftol * x_cost) return false;
    const double rel = cand_cost >= DBL_MAX ? -DBL_MAX : (x_cost - cand_cost) / model_change;
    return rel > P.lm_min_rel;
}

constexpr int kFinThreads = 256, kFinBlocks = 16;
__global__ __launch_bounds__(kFinThreads) void finalize_kernel(DevProblem P, int n_step_blocks,
                                                               unsigned long long seq) {
    double s[7] = {0, 0, 0, 0, 0, 0, 0};
    double m[5] = {0, 0, 0, 0, 0};
    // the four lists in one loop, so every list's loads are in flight together
    const int nf = P.n_fblk, nu = P.n_img * P.gram_seg, ns = P.n_chunk + P.n_gpt, nt = n_step_blocks;
    const int nmax = max(max(nf, nu), max(ns, nt));
    constexpr int kStride = kFinBlocks * kFinThreads;
#pragma unroll 2
    for (int i = blockIdx.x * kFinThreads + threadIdx.x; i < nmax; i += kStride) {
        // loads from clamped indices (unconditional, so the compiler issues
        // them all before the first use), accumulated only where in range
        const bool bf = i < nf, bu = i < nu, bs = i < ns, bt = i < nt;
        const int jf = bf ? i : 0, ju = bu ? i : 0, js = bs ? i : 0, jt = bt ? i : 0;
        // (an empty list may have no buffer: its loads are skipped, uniformly)
        double f0 = 0.0, f1 = 0.0, f2 = 0.0, u0 = 0.0, u1 = 0.0, s0 = 0.0, s1 = 0.0;
        double t0 = 0.0, t1 = 0.0, t2 = 0.0, t3 = 0.0, t4 = 0.0;
        if (nf > 0) { f0 = P.part_f[3 * jf]; f1 = P.part_f[3 * jf + 1]; f2 = P.part_f[3 * jf + 2]; }
        if (nu > 0) { u0 = P.part_u[2 * ju]; u1 = P.part_u[2 * ju + 1]; }
        if (ns > 0) { s0 = P.part_s[2 * js]; s1 = P.part_s[2 * js + 1]; }
        if (nt > 0) {
            t0 = P.part_t[kPartT * jt]; t1 = P.part_t[kPartT * jt + 1]; t2 = P.part_t[kPartT * jt + 2];
            t3 = P.part_t[kPartT * jt + 3]; t4 = P.part_t[kPartT * jt + 4];
        }
        if (bf) { s[5] += f0; s[6] += f1; m[4] = fmax(m[4], f2); }
        if (bu) { s[0] += u0; m[0] = fmax(m[0], u1); }
        if (bs) { s[1] += s0; m[1] = fmax(m[1], s1); }
        if (bt) { s[2] += t0; s[3] += t1; s[4] += t2; m[2] = fmax(m[2], t4); m[3] = fmax(m[3], t3); }
    }
    wave_sum(s);
#pragma unroll
    for (int k = 0; k < 5; ++k) m[k] = wave_max(m[k]);
    constexpr int kW = kFinThreads / 64;
    __shared__ double red[kW][12];
    __shared__ int last;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
        for (int k = 0; k < 7; ++k) red[wave][k] = s[k];
        for (int k = 0; k < 5; ++k) red[wave][7 + k] = m[k];
    }
    __syncthreads();
    if (threadIdx.x < 12) {   // one thread per scalar, waves in order
        const int k = threadIdx.x;
        double t = red[0][k];
        for (int w = 1; w < kW; ++w) t = k < 7 ? t + red[w][k] : fmax(t, red[w][k]);
        st_wt64(P.fin_part + 12 * blockIdx.x + k, t);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add((gu32_t*)P.fin_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               (unsigned)(kFinBlocks - 1);
    __syncthreads();
    if (!last) return;
    if (threadIdx.x < 12) {   // the workgroups' partials in workgroup order
        const int k = threadIdx.x;
        double t = ld_wt64(P.fin_part + k);
        for (int g = 1; g < kFinBlocks; ++g) {
            const double v = ld_wt64(P.fin_part + 12 * g + k);
            t = k < 7 ? t + v : fmax(t, v);
        }
        constexpr int kSlot[12] = {kScCost, kScXnorm2E, kScModelAcc, kScCandCost, kScStepnorm2E, kScXnorm2F,
                                   kScStepnorm2F, kScBadX, kScGmaxE, kScCandBad, kScStepBad, kScGmaxF};
        P.scal[kSlot[k]] = t;
        if (P.scal_host) P.scal_host[kSlot[k]] = t;
    }
    if (threadIdx.x == 0)   // ready for the next launch (stream order)
        __hip_atomic_store((gu32_t*)P.fin_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (P.scal_host) {
        // publish to host-mapped memory: every scalar, a system-scope fence,
        // then the sequence word the host polls (no blit, no stream sync)
        if (threadIdx.x == 12) P.scal_host[kScSolveFail] = P.scal[kScSolveFail];
        __syncthreads();   // every slot of P.scal is written
        if (threadIdx.x == 0) {
            const double acc = (P.spec_force || lm_spec_accept(P.scal, P)) ? 1.0 : 0.0;
            P.scal[kScAccept] = acc;
            P.scal_host[kScAccept] = acc;
        }
        if (threadIdx.x < 13) __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(P.scal_host + kScCount), seq,
                               __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (threadIdx.x == 0) {
        P.scal[kScAccept] = 0.0;   // a rank's partial scalars: decided after the combine
    }
}

// world > 1 over RCCL: the all-gathered per-rank scalars [world][kScMaxEnd]
// combined in rank order (sums, maxima; the replicated slots are this rank's)
// and published to host-mapped memory like finalize_kernel does at one rank,
// so the host polls a sequence word instead of copying and synchronising
__global__ void publish_gathered_kernel(DevProblem P, const double* __restrict__ g, int world,
                                        double* __restrict__ scal, double* __restrict__ host,
                                        unsigned long long seq) {
    const int k = threadIdx.x;
    if (k < kScCount && k != kScAccept) {
        double v = k < kScMaxEnd ? g[k] : scal[k];
        if (k < kScMaxEnd)
            for (int r = 1; r < world; ++r) {
                const double w = g[(size_t)r * kScMaxEnd + k];
                v = k < kScSumEnd ? v + w : fmax(v, w);
            }
        scal[k] = v;
        host[k] = v;
    }
    __syncthreads();   // the combined scalars: the accept decision (as finalize_kernel at one rank)
    if (k == 0) {
        const double acc = (P.spec_force || lm_spec_accept(scal, P)) ? 1.0 : 0.0;
        scal[kScAccept] = acc;
        host[kScAccept] = acc;
    }
    if (k < kScCount) __threadfence_system();
    __syncthreads();
    if (k == 0)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(host + kScCount), seq, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
void ba_campre(const double* extr, int n_img, CamPre* out, hipStream_t s) {
    if (n_img <= 0) return;
    hipLaunchKernelGGL(campre_kernel, dim3((n_img + 127) / 128), dim3(128), 0, s, extr, n_img, out);
    SFM_HIP(hipGetLastError());
}

// the residual model is a template parameter of every kernel that linearises
// (chunk tiles carry the model's intrinsics width: 4, RADIAL3 6)
#define SFM_BY_MODEL(P, CALL)                                  \
    do {                                                       \
        if ((P).cam_model == SFM_CAM_SNAVELY) {                \
            constexpr int CM = SFM_CAM_SNAVELY;                \
            CALL;                                              \
        } else {                                               \
            constexpr int CM = SFM_CAM_PINHOLE;                \
            CALL;                                              \
        }                                                      \
    } while (0)
#define SFM_BY_MODEL_ALL(P, CALL)                              \
    do {                                                       \
        if ((P).cam_model == SFM_CAM_RADIAL3) {                \
            constexpr int CM = SFM_CAM_RADIAL3;                \
            CALL;                                              \
        } else if ((P).cam_model == SFM_CAM_SNAVELY) {         \
            constexpr int CM = SFM_CAM_SNAVELY;                \
            CALL;                                              \
        } else {                                               \
            constexpr int CM = SFM_CAM_PINHOLE;                \
            CALL;                                              \
        }                                                      \
    } while (0)

void ba_image_gram(const DevProblem& P, const CamPre* cp, const double* intr, const double* X,
                   hipStream_t s, const double* gate) {
    if (P.n_gram_img <= 0) return;
    SFM_BY_MODEL_ALL(P, {
        hipLaunchKernelGGL((image_gram_kernel<CM, 0>), dim3(P.n_gram_img * P.gram_seg), dim3(256), 0, s, P, cp, intr,
                           X, gate);
        if constexpr (gram::SlotTable<CM>::kPasses > 1)
            hipLaunchKernelGGL((image_gram_kernel<CM, 1>), dim3(P.n_gram_img * P.gram_seg), dim3(256), 0, s, P, cp,
                               intr, X, gate);
    });
    SFM_HIP(hipGetLastError());
}

void ba_gram_rescale(const DevProblem& P, hipStream_t s) {
    if (P.n_gram_img <= 0) return;
    SFM_BY_MODEL_ALL(P, hipLaunchKernelGGL(gram_rescale_kernel<CM>, dim3(P.n_gram_img * P.gram_seg), dim3(128), 0, s, P));
    SFM_HIP(hipGetLastError());
}


void ba_fill(double* p, int64_t n, double v, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(fill_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, n, v);
    SFM_HIP(hipGetLastError());
}

void ba_segs(const SegList& L, hipStream_t s) {
    int64_t nmax = 0;
    for (int k = 0; k < L.n; ++k) nmax = std::max(nmax, L.seg[k].n);
    if (nmax <= 0) return;
    const unsigned g = (unsigned)std::min<int64_t>((nmax + 255) / 256, 2048);
    hipLaunchKernelGGL(segs_kernel, dim3(g), dim3(256), 0, s, L);
    SFM_HIP(hipGetLastError());
}

void ba_fscale(const DevProblem& P, hipStream_t s) {
    if (P.nF <= 0) return;
    hipLaunchKernelGGL(fscale_kernel, dim3((unsigned)((P.nF + 255) / 256)), dim3(256), 0, s, P);
    SFM_HIP(hipGetLastError());
}

void ba_schur(const DevProblem& P, const CamPre* cp, const double* intr, const double* X, double radius,
              hipStream_t s, unsigned long long* stamps, bool scale_e) {
    if (P.n_zbatch > 0) {
        if (scale_e)
            SFM_BY_MODEL_ALL(P, hipLaunchKernelGGL((zbatch_kernel<CM, true>), dim3(P.n_zbatch), dim3(64), 0, s, P, cp,
                                                   intr, X, radius));
        else
            SFM_BY_MODEL_ALL(P, hipLaunchKernelGGL((zbatch_kernel<CM, false>), dim3(P.n_zbatch), dim3(64), 0, s, P,
                                                   cp, intr, X, radius));
        SFM_HIP(hipGetLastError());
    }
    if (P.n_zlong > 0) {
        const size_t lds = (64 * kZStage + (size_t)P.gz_max) * sizeof(double);
        if (scale_e)
            SFM_BY_MODEL_ALL(P, {
                if (lds > 64 * 1024) set_dyn_lds((const void*)zpoint_kernel<CM, true>, lds);
                hipLaunchKernelGGL((zpoint_kernel<CM, true>), dim3(P.n_zlong), dim3(64), lds, s, P, cp, intr, X, radius);
            });
        else
            SFM_BY_MODEL_ALL(P, {
                if (lds > 64 * 1024) set_dyn_lds((const void*)zpoint_kernel<CM, false>, lds);
                hipLaunchKernelGGL((zpoint_kernel<CM, false>), dim3(P.n_zlong), dim3(64), lds, s, P, cp, intr, X, radius);
            });
        SFM_HIP(hipGetLastError());
    }
    if (P.n_group <= 0) return;
    // 64-row tiles: batches of schur4_pts(CM) points (ba_types.h) at 8 waves
    // per CU (6-point batches' LDS allows 7, and measured 9% slower)
    if (P.tile_nt == 4) {
        if (scale_e)
            SFM_BY_MODEL_ALL(P, hipLaunchKernelGGL((schur_kernel<CM, 4, schur4_pts(CM), schur4_obs(CM), true>),
                                               dim3(P.n_group), dim3(64 * schur_group(P.tile_nt)), 0, s, P, cp, intr, X, radius, stamps));
        else
            SFM_BY_MODEL_ALL(P, hipLaunchKernelGGL((schur_kernel<CM, 4, schur4_pts(CM), schur4_obs(CM)>),
                                               dim3(P.n_group), dim3(64 * schur_group(P.tile_nt)), 0, s, P, cp, intr, X, radius, stamps));
    } else {
        if (scale_e)
            SFM_BY_MODEL_ALL(P, hipLaunchKernelGGL((schur_kernel<CM, 5, kSubPts, kSubObs, true>),
                                               dim3(P.n_group), dim3(64 * schur_group(P.tile_nt)), 0, s, P, cp, intr, X, radius, stamps));
        else
            SFM_BY_MODEL_ALL(P, hipLaunchKernelGGL((schur_kernel<CM, 5, kSubPts, kSubObs>), dim3(P.n_group),
                                               dim3(64 * schur_group(P.tile_nt)), 0, s, P, cp, intr, X, radius, stamps));
    }
    SFM_HIP(hipGetLastError());
}

void ba_reduce(const DevProblem& P, bool vectors_only, hipStream_t s) {
    if (P.n_targets <= 0 && P.n_zero <= 0) return;
    const int per_block = 4 / P.red_waves, nb = (P.n_targets + per_block - 1) / per_block;
    const bool split = P.red_split != 0;   // SFM_CTX_BA_SPLIT_REDUCE: three launches
    const int nz = (P.n_zero + 15) / 16;   // zero-list workgroups, last in the grid
    if (P.n_long > 0 && !split) {
        hipLaunchKernelGGL(reduce_kernel<true>, dim3(nb + P.n_lseg + nz), dim3(256), 0, s, P, vectors_only ? 1 : 0,
                           nb, nb + P.n_lseg);
        SFM_HIP(hipGetLastError());
    } else {
        hipLaunchKernelGGL(reduce_kernel<false>, dim3(nb + nz), dim3(256), 0, s, P, vectors_only ? 1 : 0, nb, nb);
        SFM_HIP(hipGetLastError());
    }
    if (P.n_long > 0 && split) {
        hipLaunchKernelGGL(reduce_seg_kernel, dim3(P.n_lseg), dim3(256), 0, s, P, vectors_only ? 1 : 0);
        SFM_HIP(hipGetLastError());
        hipLaunchKernelGGL(reduce_long_kernel, dim3(P.n_long), dim3(64), 0, s, P, vectors_only ? 1 : 0);
        SFM_HIP(hipGetLastError());
    }
    // product terms (general points) land on the matrix and rhs targets
    if (P.n_gpt > 0 && !vectors_only) {
        hipLaunchKernelGGL(preduce_kernel, dim3((P.n_targets + 3) / 4), dim3(256), 0, s, P);
        SFM_HIP(hipGetLastError());
        if (P.n_plong > 0) {
            hipLaunchKernelGGL(preduce_seg_kernel, dim3(P.n_plseg), dim3(256), 0, s, P);
            SFM_HIP(hipGetLastError());
            hipLaunchKernelGGL(preduce_long_kernel, dim3(P.n_plong), dim3(64), 0, s, P);
            SFM_HIP(hipGetLastError());
        }
    }
}

int reduce_long_threshold() { return kLongTerms; }
int preduce_long_threshold() { return kLongPTerms; }

size_t solve_window_doubles(const DevProblem& P) {
    const size_t Dp = P.D + 1;
    return Dp * Dp * 36 + (size_t)P.nintr * Dp * 24 + 16 * (size_t)P.nintr * P.nintr + Dp * 6 +
           4 * (size_t)P.nintr;
}

size_t solve_lds_bytes(const DevProblem& P, bool* use_lds) {
    const size_t small = (2 + (size_t)(P.D + 1) * 6) * sizeof(double);
    const size_t full = small + solve_window_doubles(P) * sizeof(double);
    *use_lds = full <= 150 * 1024;
    return *use_lds ? full : small;
}

void ba_solve(const DevProblem& P, double radius, hipStream_t s) {
    bool lds = false;
    const size_t bytes = solve_lds_bytes(P, &lds);
    SFM_REQUIRE(bytes <= 160 * 1024, SFM_ERR_UNSUPPORTED, "RCS band too wide (D=%d)", P.D);
    if (bytes > 64 * 1024) set_dyn_lds((const void*)solve_kernel, bytes);
    hipLaunchKernelGGL(solve_kernel, dim3(1), dim3(256), bytes, s, P, radius, lds ? 1 : 0);
    SFM_HIP(hipGetLastError());
}

int ba_cand_blocks(const DevProblem& P) {
    return std::max(1, (P.n_img + P.n_intr + kCandThreads - 1) / kCandThreads);
}
void ba_cand(const DevProblem& P, const double* extr, const double* intr, double* cand_extr,
             double* cand_intr, CamPre* cand_cp, hipStream_t s) {
    hipLaunchKernelGGL(cand_kernel, dim3(P.n_fblk), dim3(kCandThreads), 0, s, P, extr, intr,
                       cand_extr, cand_intr, cand_cp);
    SFM_HIP(hipGetLastError());
}

int ba_step_blocks(const DevProblem& P) { return P.n_chunk + (P.n_gpt + kGStepThreads - 1) / kGStepThreads; }

void ba_step(const DevProblem& P, const CamPre* cp, const double* intr, const CamPre* cp_cand,
             const double* intr_cand, const double* X, double* X_cand, double radius, hipStream_t s) {
    if (P.n_chunk > 0) {
        const int split = P.step_split;
        const int threads = std::min(kStepThreads, (P.chunk_pts_max * split + 63) / 64 * 64);
        SFM_REQUIRE(P.chunk_pts_max * split <= threads, SFM_ERR_UNSUPPORTED, "step kernel: chunk exceeds the workgroup");
        auto go = [&](auto tag) {
            constexpr int SP = decltype(tag)::value;
            SFM_BY_MODEL_ALL(P, hipLaunchKernelGGL((step_kernel<CM, SP>), dim3(P.n_chunk), dim3(threads), 0, s, P,
                                                   cp, intr, cp_cand, intr_cand, X, X_cand, radius));
        };
        if (split == 8) go(std::integral_constant<int, 8>{});
        else if (split == 4) go(std::integral_constant<int, 4>{});
        else if (split == 2) go(std::integral_constant<int, 2>{});
        else go(std::integral_constant<int, 1>{});
        SFM_HIP(hipGetLastError());
    }
    if (P.n_gpt > 0) {
        const int nb = (P.n_gpt + kGStepThreads - 1) / kGStepThreads;
        SFM_BY_MODEL_ALL(P, hipLaunchKernelGGL(step_general_kernel<CM>, dim3(nb), dim3(kGStepThreads), 0, s, P, cp, intr,
                                           cp_cand, intr_cand, X, X_cand, radius));
        SFM_HIP(hipGetLastError());
    }
}

void ba_finalize(const DevProblem& P, hipStream_t s, unsigned long long seq) {
    hipLaunchKernelGGL(finalize_kernel, dim3(kFinBlocks), dim3(kFinThreads), 0, s, P, ba_step_blocks(P), seq);
    SFM_HIP(hipGetLastError());
}

void ba_publish_gathered(const DevProblem& P, const double* gathered, int world, double* scal, double* scal_host,
                         hipStream_t s, unsigned long long seq) {
    hipLaunchKernelGGL(publish_gathered_kernel, dim3(1), dim3(64), 0, s, P, gathered, world, scal, scal_host, seq);
    SFM_HIP(hipGetLastError());
}

}  // namespace sfm
