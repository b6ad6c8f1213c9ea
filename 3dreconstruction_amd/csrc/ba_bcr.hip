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
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "ba_bcr.h"
#include "common.h"

namespace sfm {
namespace {

constexpr int M = kBcrM;      // 64
constexpr int LD = M + 1;     // LDS row stride (bank spread)
constexpr int NT = 256;

__device__ __forceinline__ double clampd(double v, double lo, double hi) { return fmin(fmax(v, lo), hi); }

// ---- dense helpers on LDS tiles, 256 threads --------------------------------
// in-place lower Cholesky of a 64x64 tile; returns false on a non-positive pivot
// `bad` lives in the dynamic LDS region (a static __shared__ would misalign it)
__device__ bool chol64(double* A, double* bad) {
    if (threadIdx.x == 0) bad[0] = 0.0;
    __syncthreads();
    for (int k = 0; k < M; ++k) {
        if (threadIdx.x == 0) {
            const double d = A[k * LD + k];
            if (!(d > 0.0)) bad[0] = 1.0;
            A[k * LD + k] = sqrt(d);
        }
        __syncthreads();
        const double inv = 1.0 / A[k * LD + k];
        for (int i = k + 1 + threadIdx.x; i < M; i += NT) A[i * LD + k] *= inv;
        __syncthreads();
        // trailing lower update: A[i][j] -= A[i][k] A[j][k], k < j <= i
        const int n = M - 1 - k;
        for (int e = threadIdx.x; e < n * n; e += NT) {
            const int i = k + 1 + e / n, j = k + 1 + e % n;
            if (j <= i) A[i * LD + j] -= A[i * LD + k] * A[j * LD + k];
        }
        __syncthreads();
    }
    return bad[0] == 0.0;
}

// B <- L^-1 B for B [64][nc] with row stride ldb (lower L from chol64)
__device__ void trsm64(const double* L, double* B, int nc, int ldb) {
    for (int k = 0; k < M; ++k) {
        const double inv = 1.0 / L[k * LD + k];
        for (int c = threadIdx.x; c < nc; c += NT) B[k * ldb + c] *= inv;
        __syncthreads();
        const int n = M - 1 - k;
        for (int e = threadIdx.x; e < n * nc; e += NT) {
            const int i = k + 1 + e / nc, c = e % nc;
            B[i * ldb + c] -= L[i * LD + k] * B[k * ldb + c];
        }
        __syncthreads();
    }
}

// B <- L^-T B
__device__ void trsm64_t(const double* L, double* B, int nc, int ldb) {
    for (int k = M - 1; k >= 0; --k) {
        const double inv = 1.0 / L[k * LD + k];
        for (int c = threadIdx.x; c < nc; c += NT) B[k * ldb + c] *= inv;
        __syncthreads();
        for (int e = threadIdx.x; e < k * nc; e += NT) {
            const int i = e / nc, c = e % nc;
            B[i * ldb + c] -= L[k * LD + i] * B[k * ldb + c];
        }
        __syncthreads();
    }
}

__device__ void load64(double* dst, const double* src) {  // global [64][64] -> LDS [64][LD]
    for (int e = threadIdx.x; e < M * M; e += NT) dst[(e / M) * LD + e % M] = src[e];
}
__device__ void store64(double* dst, const double* src) {
    for (int e = threadIdx.x; e < M * M; e += NT) dst[e] = src[(e / M) * LD + e % M];
}

// ---- pack: band (6x6 blocks) -> 64x64 super-blocks, D^2 added, identity pad --
__global__ void bcr_pack_kernel(BcrArgs b, DevProblem P, double radius) {
    const int I = blockIdx.x;
    double* A = b.A + (size_t)I * M * M;
    double* Cm = b.C + (size_t)I * M * M;
    double* R = b.R + (size_t)I * M * b.nrhs;
    const int c0 = I * b.K, nreal = min(b.K, P.ncam - c0) * 6;
    const int Dp = P.D + 1;
    for (int e = threadIdx.x; e < M * M; e += NT) {
        const int r = e / M, c = e % M;
        double a = 0.0, cc = 0.0;
        if (r < nreal) {
            const int ci = c0 + r / 6;
            // A: block (ci, cj) with cj in this super-block, cj <= ci (lower), mirror upper
            if (c < nreal) {
                const int cj = c0 + c / 6;
                const int hi = max(ci, cj), lo = min(ci, cj);
                const int d = hi - lo;
                if (d <= P.D) {
                    const int rr = ci >= cj ? r % 6 : c % 6, cc2 = ci >= cj ? c % 6 : r % 6;
                    a = P.Sband[((size_t)hi * Dp + d) * 36 + rr * 6 + cc2];
                }
                if (r == c) {
                    const double lm = sqrt(clampd(P.cnF[6LL * ci + r % 6], P.min_diag, P.max_diag) / radius);
                    a += lm * lm;
                }
            }
            // C: block (ci, cj) with cj in the previous super-block
            if (I > 0 && c / 6 < b.K) {   // the previous super-block is always full
                const int cj = c0 - b.K + c / 6;
                const int d = ci - cj;
                if (d >= 1 && d <= P.D) cc = P.Sband[((size_t)ci * Dp + d) * 36 + (r % 6) * 6 + c % 6];
            }
        } else if (r == c) {
            a = 1.0;  // padding: identity
        }
        A[e] = a;
        Cm[e] = cc;
    }
    // R: column 0 = rhs, columns 1 + 4k + a = arrow (intr k, row a) transposed
    for (int e = threadIdx.x; e < M * b.nrhs; e += NT) {
        const int r = e / b.nrhs, c = e % b.nrhs;
        double v = 0.0;
        if (r < nreal) {
            const int ci = c0 + r / 6;
            if (c == 0) v = P.rhs[6LL * ci + r % 6];
            else if (c - 1 < 4 * P.nintr) {
                const int k = (c - 1) / 4, a = (c - 1) % 4;
                v = P.Sarrow[((size_t)k * P.ncam + ci) * 24 + a * 6 + r % 6];
            }
        }
        R[e] = v;
    }
}

// ---- level l: factor every odd super-block, W = L^-1 C, z = L^-1 R -----------
__global__ __launch_bounds__(NT) void bcr_factor_kernel(BcrArgs b, int s) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* A = sm;                 // [64][LD]
    double* B = A + M * LD;         // [64][LD]
    double* R = B + M * LD;         // [64][nrhs+1]
    const int ldr = b.nrhs + 1;
    double* flag = R + M * ldr;     // [2]
    const int i = s + 2 * s * blockIdx.x;   // odd at this level
    if (i >= b.N) return;
    const int r = i + s;
    load64(A, b.A + (size_t)i * M * M);
    __syncthreads();
    if (!chol64(A, flag) && threadIdx.x == 0) b.fail[0] = 1.0;
    store64(b.L + (size_t)i * M * M, A);
    // W_l = L^-1 C_i   (C_i = block (i, i-s))
    load64(B, b.C + (size_t)i * M * M);
    __syncthreads();
    trsm64(A, B, M, LD);
    store64(b.Wl + (size_t)i * M * M, B);
    __syncthreads();
    if (r < b.N) {  // W_r = L^-1 C_r'   (C_r = block (r, i))
        const double* Cr = b.C + (size_t)r * M * M;
        for (int e = threadIdx.x; e < M * M; e += NT) B[(e % M) * LD + e / M] = Cr[e];
        __syncthreads();
        trsm64(A, B, M, LD);
        store64(b.Wr + (size_t)i * M * M, B);
        __syncthreads();
    }
    const double* Rg = b.R + (size_t)i * M * b.nrhs;
    for (int e = threadIdx.x; e < M * b.nrhs; e += NT) R[(e / b.nrhs) * ldr + e % b.nrhs] = Rg[e];
    __syncthreads();
    trsm64(A, R, b.nrhs, ldr);
    double* Z = b.Z + (size_t)i * M * b.nrhs;
    for (int e = threadIdx.x; e < M * b.nrhs; e += NT) Z[e] = R[(e / b.nrhs) * ldr + e % b.nrhs];
}

// ---- level l: update every even super-block from its odd neighbours ---------
// A_j -= Wr_{j-s}' Wr_{j-s} + Wl_{j+s}' Wl_{j+s};  R_j -= Wr' z + Wl' z;
// new coupling C_j (block (j, j-2s)) = -Wr_{j-s}' Wl_{j-s}
__global__ __launch_bounds__(NT) void bcr_update_kernel(BcrArgs b, int s) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* X = sm;            // [64][LD]
    double* Y = X + M * LD;    // [64][LD]
    const int j = 2 * s * blockIdx.x;
    if (j >= b.N) return;
    const int il = j - s, ir = j + s;   // odd neighbours
    double* Aj = b.A + (size_t)j * M * M;
    double* Rj = b.R + (size_t)j * M * b.nrhs;
    const int tr = threadIdx.x / 16, tc = threadIdx.x % 16;   // 4x4 output blocks
    double acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[a][c] = 0.0;
    auto gemm_tn = [&](const double* P1, const double* P2) {  // acc += P1' P2 (LDS)
        for (int k = 0; k < M; ++k) {
            double x[4], y[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) { x[a] = P1[k * LD + 4 * tr + a]; y[a] = P2[k * LD + 4 * tc + a]; }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[a][c] += x[a] * y[c];
        }
    };
    if (il >= 0) {
        load64(X, b.Wr + (size_t)il * M * M);
        __syncthreads();
        gemm_tn(X, X);
        __syncthreads();
    }
    if (ir < b.N) {
        load64(Y, b.Wl + (size_t)ir * M * M);
        __syncthreads();
        gemm_tn(Y, Y);
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) Aj[(4 * tr + a) * M + 4 * tc + c] -= acc[a][c];
    // rhs
    for (int e = threadIdx.x; e < M * b.nrhs; e += NT) {
        const int row = e / b.nrhs, c = e % b.nrhs;
        double v = 0.0;
        if (il >= 0) {
            const double* W = b.Wr + (size_t)il * M * M;
            const double* Z = b.Z + (size_t)il * M * b.nrhs;
            for (int k = 0; k < M; ++k) v += W[k * M + row] * Z[k * b.nrhs + c];
        }
        if (ir < b.N) {
            const double* W = b.Wl + (size_t)ir * M * M;
            const double* Z = b.Z + (size_t)ir * M * b.nrhs;
            for (int k = 0; k < M; ++k) v += W[k * M + row] * Z[k * b.nrhs + c];
        }
        Rj[e] -= v;
    }
    // new coupling to j - 2s
    if (il >= 0 && j - 2 * s >= 0) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[a][c] = 0.0;
        load64(X, b.Wr + (size_t)il * M * M);
        load64(Y, b.Wl + (size_t)il * M * M);
        __syncthreads();
        gemm_tn(X, Y);
        double* Cj = b.C + (size_t)j * M * M;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int c = 0; c < 4; ++c) Cj[(4 * tr + a) * M + 4 * tc + c] = -acc[a][c];
    }
}

// ---- top: super-block 0 alone; y_0 = A_0^-1 R_0 -------------------------------
__global__ __launch_bounds__(NT) void bcr_top_kernel(BcrArgs b) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* A = sm;
    double* R = A + M * LD;
    const int ldr = b.nrhs + 1;
    double* flag = R + M * ldr;
    load64(A, b.A);
    for (int e = threadIdx.x; e < M * b.nrhs; e += NT) R[(e / b.nrhs) * ldr + e % b.nrhs] = b.R[e];
    __syncthreads();
    if (!chol64(A, flag) && threadIdx.x == 0) b.fail[0] = 1.0;
    trsm64(A, R, b.nrhs, ldr);
    trsm64_t(A, R, b.nrhs, ldr);
    for (int e = threadIdx.x; e < M * b.nrhs; e += NT) b.Y[e] = R[(e / b.nrhs) * ldr + e % b.nrhs];
}

// ---- back substitution at level l: y_i = L_i^-T (z_i - Wl y_l - Wr y_r) -------
__global__ __launch_bounds__(NT) void bcr_back_kernel(BcrArgs b, int s) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* A = sm;
    double* R = A + M * LD;
    const int ldr = b.nrhs + 1;
    const int i = s + 2 * s * blockIdx.x;
    if (i >= b.N) return;
    const int l = i - s, r = i + s;
    load64(A, b.L + (size_t)i * M * M);
    const double* Z = b.Z + (size_t)i * M * b.nrhs;
    const double* Wl = b.Wl + (size_t)i * M * M;
    const double* Wr = b.Wr + (size_t)i * M * M;
    const double* Yl = b.Y + (size_t)l * M * b.nrhs;
    const double* Yr = b.Y + (size_t)r * M * b.nrhs;
    for (int e = threadIdx.x; e < M * b.nrhs; e += NT) {
        const int row = e / b.nrhs, c = e % b.nrhs;
        double v = Z[e];
        for (int k = 0; k < M; ++k) v -= Wl[row * M + k] * Yl[k * b.nrhs + c];
        if (r < b.N)
            for (int k = 0; k < M; ++k) v -= Wr[row * M + k] * Yr[k * b.nrhs + c];
        R[row * ldr + c] = v;
    }
    __syncthreads();
    trsm64_t(A, R, b.nrhs, ldr);
    double* Y = b.Y + (size_t)i * M * b.nrhs;
    for (int e = threadIdx.x; e < M * b.nrhs; e += NT) Y[e] = R[(e / b.nrhs) * ldr + e % b.nrhs];
}

// ---- bordered arrow: corner system and final y_F --------------------------------
// M_c = S_corner + D^2 - sum_I B_I' Yb_I ; v = rhs_c - sum_I B_I' y0_I
__global__ __launch_bounds__(NT) void bcr_corner_kernel(BcrArgs b, DevProblem P, double radius) {
    const int na4 = 4 * P.nintr;
    __shared__ double Mc[16 * 16 + 16];
    __shared__ double red[NT];
    const int nent = na4 * na4 + na4;
    for (int q = 0; q < nent; ++q) {
        // q < na4*na4: (a, c) -> sum_I sum_row B_I[row][a] Yb_I[row][c]; else v_a
        const int a = q < na4 * na4 ? q / na4 : q - na4 * na4;
        const int c = q < na4 * na4 ? q % na4 : -1;
        double v = 0.0;
        for (int e = threadIdx.x; e < b.N * M; e += NT) {
            const int I = e / M, row = e % M;
            const double* R0 = b.R0 + ((size_t)I * M + row) * b.nrhs;  // original R (B in cols 1..)
            const double* Y = b.Y + ((size_t)I * M + row) * b.nrhs;
            v += R0[1 + a] * (c >= 0 ? Y[1 + c] : Y[0]);
        }
        red[threadIdx.x] = v;
        __syncthreads();
        for (int o = NT / 2; o > 0; o >>= 1) {
            if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            if (c >= 0) {
                double m = P.Scorner[(((size_t)(a / 4) * P.nintr + c / 4) * 16) + (a % 4) * 4 + c % 4];
                if (a == c) {
                    const double lm = sqrt(clampd(P.cnF[P.nb + a], P.min_diag, P.max_diag) / radius);
                    m += lm * lm;
                }
                Mc[a * 16 + c] = m - red[0];
            } else {
                Mc[256 + a] = P.rhs[P.nb + a] - red[0];
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        // dense Cholesky solve of the corner (<= 16 x 16)
        bool ok = true;
        for (int j = 0; j < na4; ++j) {
            double d = Mc[j * 16 + j];
            for (int k = 0; k < j; ++k) d -= Mc[j * 16 + k] * Mc[j * 16 + k];
            if (!(d > 0.0)) ok = false;
            d = sqrt(d);
            Mc[j * 16 + j] = d;
            for (int i = j + 1; i < na4; ++i) {
                double t = Mc[i * 16 + j];
                for (int k = 0; k < j; ++k) t -= Mc[i * 16 + k] * Mc[j * 16 + k];
                Mc[i * 16 + j] = t / d;
            }
        }
        double* v = Mc + 256;
        for (int i = 0; i < na4; ++i) {
            double t = v[i];
            for (int k = 0; k < i; ++k) t -= Mc[i * 16 + k] * v[k];
            v[i] = t / Mc[i * 16 + i];
        }
        for (int i = na4 - 1; i >= 0; --i) {
            double t = v[i];
            for (int k = i + 1; k < na4; ++k) t -= Mc[k * 16 + i] * v[k];
            v[i] = t / Mc[i * 16 + i];
            P.yF[P.nb + i] = v[i];
        }
        if (!ok) b.fail[0] = 1.0;
    }
}

// y_band = y0 - Yb x_c, written in F order; also the solve-failure flag
__global__ void bcr_final_kernel(BcrArgs b, DevProblem P) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e == 0) P.scal[kScSolveFail] = b.fail[0];
    if (e >= P.nb) return;
    const int ci = (int)(e / 6), I = ci / b.K, row = (ci - I * b.K) * 6 + (int)(e % 6);
    const double* Y = b.Y + ((size_t)I * M + row) * b.nrhs;
    double v = Y[0];
    for (int a = 0; a < 4 * P.nintr; ++a) v -= Y[1 + a] * P.yF[P.nb + a];
    P.yF[e] = v;
}

}  // namespace

bool bcr_supported(const DevProblem& P) { return P.D <= kBcrK && P.ncam > 0 && 1 + 4 * P.nintr <= 32; }

void bcr_setup(BcrArgs& b, const DevProblem& P) {
    b.K = kBcrK;
    b.N = (P.ncam + b.K - 1) / b.K;
    b.nrhs = ((1 + 4 * P.nintr) + 7) / 8 * 8;
}

size_t bcr_doubles(const BcrArgs& b) {
    const size_t mm = (size_t)b.N * M * M, mr = (size_t)b.N * M * b.nrhs;
    return 5 * mm + 4 * mr + 8;  // A C L Wl Wr | R R0 Z Y | fail
}

void bcr_bind(BcrArgs& b, double* base) {
    const size_t mm = (size_t)b.N * M * M, mr = (size_t)b.N * M * b.nrhs;
    b.A = base; b.C = b.A + mm; b.L = b.C + mm; b.Wl = b.L + mm; b.Wr = b.Wl + mm;
    b.R = b.Wr + mm; b.R0 = b.R + mr; b.Z = b.R0 + mr; b.Y = b.Z + mr; b.fail = b.Y + mr;
}

void bcr_solve(const BcrArgs& b, const DevProblem& P, double radius, hipStream_t s) {
    SFM_HIP(hipMemsetAsync(b.fail, 0, sizeof(double), s));
    hipLaunchKernelGGL(bcr_pack_kernel, dim3(b.N), dim3(NT), 0, s, b, P, radius);
    SFM_HIP(hipGetLastError());
    SFM_HIP(hipMemcpyAsync(b.R0, b.R, (size_t)b.N * M * b.nrhs * sizeof(double), hipMemcpyDeviceToDevice, s));
    const size_t lds_f = (2 * M * LD + M * (b.nrhs + 1) + 2) * sizeof(double);
    const size_t lds_u = 2 * M * LD * sizeof(double);
    const size_t lds_t = (M * LD + M * (b.nrhs + 1) + 2) * sizeof(double);
    static bool attr = false;
    if (!attr) {
        SFM_HIP(hipFuncSetAttribute((const void*)bcr_factor_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_f));
        SFM_HIP(hipFuncSetAttribute((const void*)bcr_update_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_u));
        SFM_HIP(hipFuncSetAttribute((const void*)bcr_top_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(M * LD + M * 33 + 2) * 8));
        SFM_HIP(hipFuncSetAttribute((const void*)bcr_back_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(M * LD + M * 33 + 2) * 8));
        attr = true;
    }
    int s_top = 1;
    for (int stride = 1; stride < b.N; stride *= 2) {
        const int n_odd = (b.N - stride + 2 * stride - 1) / (2 * stride);
        const int n_even = (b.N + 2 * stride - 1) / (2 * stride);
        hipLaunchKernelGGL(bcr_factor_kernel, dim3(n_odd), dim3(NT), lds_f, s, b, stride);
        SFM_HIP(hipGetLastError());
        hipLaunchKernelGGL(bcr_update_kernel, dim3(n_even), dim3(NT), lds_u, s, b, stride);
        SFM_HIP(hipGetLastError());
        s_top = stride * 2;
    }
    hipLaunchKernelGGL(bcr_top_kernel, dim3(1), dim3(NT), lds_t, s, b);
    SFM_HIP(hipGetLastError());
    for (int stride = s_top / 2; stride >= 1; stride /= 2) {
        if (stride >= b.N) continue;
        const int n_odd = (b.N - stride + 2 * stride - 1) / (2 * stride);
        hipLaunchKernelGGL(bcr_back_kernel, dim3(n_odd), dim3(NT), lds_t, s, b, stride);
        SFM_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(bcr_corner_kernel, dim3(1), dim3(NT), 0, s, b, P, radius);
    SFM_HIP(hipGetLastError());
    hipLaunchKernelGGL(bcr_final_kernel, dim3((unsigned)((P.nb + 255) / 256 + 1)), dim3(256), 0, s, b, P);
    SFM_HIP(hipGetLastError());
}

}  // namespace sfm
