// All-pairs 128-D SIFT descriptor matching on CDNA4 (gfx950).
//
// Reference path: src/sparseBuilder/sparseBuilder.cpp:809-1023 (match(),
// Matcher_Regions(0.8, BRUTE_FORCE_L2) :919-921, fDistRatio :812) over the
// exhaustive pair list of matchPair() :758-807; and the legacy exact matcher
// src/frame/LocalFrame.h:31-47 / GlobalFrame.h:22-43 (BFMatcher crossCheck).
//
// Design:
//   * descriptors are uint8 128-D; they are stored once in HBM as int8
//     a' = a - 128 (translation keeps |a-b|^2) with |a'|^2 per row, so the
//     distance matrix is an exact integer contraction on the i8 MFMA
//     (v_mfma_i32_32x32x32_i8, int32 accumulate): |a'|^2+|b'|^2-2a'.b'.
//   * one workgroup = 4 waves of kCT x 32 queries of image J against all of image I;
//     each wave keeps its kCT x 32 queries' B fragments in VGPRs and streams the
//     database in 32-row MFMA tiles; the C tile has the database row on the
//     registers and the query on the lane, so the top-2 update is lane-local:
//     key = ((|d'|^2 << 8) | row&255) - 512 * dot, two keys x, y per update:
//     b2 = min(med3(b1,x,y), b2), b1 = min3(b1,x,y) (2.25 VALU ops per
//     distance including the key), merged with the running
//     (value, index) state every 256 rows; lowest index wins ties.
//   * the ratio test d1 < fl32(ratio^2) * d2 and the result write are fused
//     into the epilogue; nothing but (idx, d1) per query leaves the chip.
//   * blockIdx -> (pair, query block) is XCD-aware: the query blocks of one
//     pair, and consecutive pairs (which share image I), land on one XCD so
//     the database image is served from that XCD's L2.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <type_traits>
#include <vector>

#include "cascade.h"
#include "common.h"

namespace sfm {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kWaves = 4;          // waves per workgroup
constexpr int kThreads = 64 * kWaves;
constexpr int kCT = 4;             // 32-query column tiles per wave (even; 4: 200 VGPRs, 2 waves/SIMD)
static_assert(kCT % 2 == 0 && kCT >= 2, "the epilogue walks column tiles in pairs");
constexpr int kQW = 32 * kCT;      // queries per wave
constexpr int kQB = kWaves * kQW;  // queries per workgroup
constexpr int kRowPad = kQB > 256 ? kQB : 256;  // rows of every image padded to this multiple
constexpr int kStage = 128;        // database rows per LDS stage (kRowPad multiple of it)
static_assert(kStage == 128 || kStage == 256, "merge windows are 256 rows");
#ifndef MATCH_TILE_UNROLL
#define MATCH_TILE_UNROLL 1        // tile-loop unroll (tests/test_match_isa.py builds 1 and 2)
#endif
// Measured and not kept (the code is in git history):
// a software-pipelined tile loop (two accumulator sets), 8-wave ping-pong
// workgroups (waves w and w + 4 half a tile apart), 256-row stages, one
// [2][...] stage array (the waitcnt pass then waited for the next stage's
// LDS DMA at every tile loop head).

// u8 -> int8 (a ^ 0x80 == a - 128), per-row |a'|^2 and the packed key base.
__global__ void prep_kernel(uint8_t* __restrict__ d, int32_t* __restrict__ nrm,
                            int32_t* __restrict__ ntr, const int64_t* __restrict__ row_img_start,
                            const int32_t* __restrict__ row_valid, int64_t n_rows) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= n_rows) return;
    uint16_t* row = reinterpret_cast<uint16_t*>(d + r * 128);
    uint16_t v = row[lane];
    v ^= 0x8080;
    row[lane] = v;
    const int lo = (int)(int8_t)(v & 0xff), hi = (int)(int8_t)(v >> 8);
    int s = lo * lo + hi * hi;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) {
        const bool valid = row_valid[r] != 0;
        nrm[r] = s;
        const int64_t local = r - row_img_start[r];
        ntr[r] = valid ? ((s << 8) | (int)(local & 255)) : INT_MAX;
    }
}

// lowered to v_min3_i32 / v_med3_i32 (SIISelLowering's min/max combines)
__device__ __forceinline__ int min3i(int a, int b, int c) { return min(min(a, b), c); }
__device__ __forceinline__ int med3i(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }
// the value unchanged, hidden from the optimiser (an empty asm: no
// instruction is emitted, so there is nothing for the hazard recognizer)
__device__ __forceinline__ int opaque(int v) {
    asm("" : "+v"(v));
    return v;
}

struct Top2 {
    int g1v, g1i, g2v;
};

__device__ __forceinline__ void merge_tile(Top2& g, int b1, int b2, int base) {
    // tile keys: value = key >> 8, index = base + (key & 255); tiles arrive in
    // increasing index order so strict '<' keeps the lower index on ties.
    const int t1v = b1 >> 8, t2v = b2 >> 8;
    const int t1i = base + (b1 & 255);
    if (t1v < g.g1v) {
        g.g2v = min(g.g1v, t2v);
        g.g1v = t1v;
        g.g1i = t1i;
    } else {
        g.g2v = min(g.g2v, t1v);
    }
}

__device__ __forceinline__ void merge_lanes(Top2& g) {
    const int o1v = __shfl_xor(g.g1v, 32), o1i = __shfl_xor(g.g1i, 32),
              o2v = __shfl_xor(g.g2v, 32);
    const bool other_first = o1v < g.g1v || (o1v == g.g1v && o1i < g.g1i);
    if (other_first) {
        g.g2v = min(g.g1v, o2v);
        g.g1v = o1v;
        g.g1i = o1i;
    } else {
        g.g2v = min(g.g2v, o1v);
    }
}

struct MatchArgs {
    const int8_t* desc;        // padded rows x 128 (int8, a - 128)
    const int32_t* nrm;        // |a'|^2 per padded row
    const int32_t* ntr;        // (|a'|^2 << 8) | (row & 255); INT_MAX for pad rows
    const int64_t* img_row0;   // first padded row of each image
    const int32_t* img_n;      // valid rows per image
    const int32_t* pairs;      // (I, J) per pair of this batch
    int32_t n_pairs;
    int32_t qblocks;           // query blocks per pair (max over the batch)
    int32_t swap;              // 0: queries = J, database = I; 1: queries = I, db = J
    int32_t ratio_test;        // apply d1 < r2*d2 (RATIO mode)
    int32_t kmul;              // -512 (runtime, keeps v_mad_i32_i24)
    float r2;
    int64_t out_stride;        // entries per pair in the outputs
    int32_t* out_idx;          // [n_pairs][out_stride]
    int32_t* out_d;            // [n_pairs][out_stride]
};

// kRatio = false (MUTUAL's two nearest-neighbour passes): only the nearest
// key is tracked (min3 over two keys, 1.5 VALU per distance).
template <bool kRatio>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void match_top2_kernel(MatchArgs a) {
    // XCD-aware bijective remap of the flat workgroup id (guide §5 T1):
    // blocks b and b+8 share an XCD, so give each XCD a contiguous range of
    // work items (pair-major, query block minor).
    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int work = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int pair = work / a.qblocks;
    const int qblk = work - pair * a.qblocks;
    if (pair >= a.n_pairs) return;
    const int I = a.pairs[2 * pair], J = a.pairs[2 * pair + 1];
    const int db_img = a.swap ? J : I, q_img = a.swap ? I : J;
    const int n_db = a.img_n[db_img], n_q = a.img_n[q_img];
    if (qblk * kQB >= n_q) return;

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int h = lane >> 5, c = lane & 31;
    const int64_t q_row0 = a.img_row0[q_img] + qblk * kQB + wave * kQW;
    const int64_t db_row0 = a.img_row0[db_img];

    // B fragments: 2 column tiles x 4 k-steps, lane holds bytes [64h+16s, +16)
    // of query row c (k assignment shared with A; MFMA pairs equal slots).
    v4i bq[kCT][4];
#pragma unroll
    for (int t = 0; t < kCT; ++t) {
        const v4i* src = reinterpret_cast<const v4i*>(a.desc + (q_row0 + 32 * t + c) * 128 + 64 * h);
#pragma unroll
        for (int s = 0; s < 4; ++s) bq[t][s] = src[s];
    }

    Top2 g[kCT];
#pragma unroll
    for (int t = 0; t < kCT; ++t) { g[t].g1v = INT_MAX; g[t].g1i = -1; g[t].g2v = INT_MAX; }

    // Database rows are staged once per workgroup through LDS (double-buffered
    // kStage-row stages filled by global_load_lds, 16 B per lane), instead of
    // every wave loading its fragments from L2.  The LDS image is lane-linear;
    // bank conflicts of the 32-rows-one-chunk fragment reads are removed by
    // storing logical 16-byte chunk k of row r at slot k ^ (r & 7) (the XOR is
    // applied to the global SOURCE address, and again on the read).
    // The two stage buffers are separate LDS objects and the stage loop is
    // unrolled by two, so every fragment read names one of them: the waitcnt
    // pass can then tell that the reads of one stage do not alias the LDS-DMA
    // writes of the next and does not wait for those at the tile loop's head.
    __shared__ __attribute__((aligned(16))) int8_t sA0[kStage * 128], sA1[kStage * 128];
    __shared__ __attribute__((aligned(16))) int32_t sN0[kStage], sN1[kStage];
    auto issue_to = [&](int8_t* dA, int32_t* dN, int row_base) {
#pragma unroll
        for (int q = 0; q < kStage * 8 / kThreads; ++q) {
            const int L = q * kThreads + wave * 64 + lane;     // 16-byte slot in the stage
            const int r = L >> 3, k = (L & 7) ^ (r & 7);
            const int8_t* src = a.desc + (db_row0 + row_base + r) * 128 + k * 16;
            __builtin_amdgcn_global_load_lds(src, dA + (q * kThreads + wave * 64) * 16, 16, 0, 0);
        }
        if (wave == 0) {
#pragma unroll
            for (int q = 0; q < kStage / 64; ++q)
                __builtin_amdgcn_global_load_lds(a.ntr + db_row0 + row_base + q * 64 + lane, dN + q * 64, 4, 0, 0);
        }
    };
    // (256-row merge windows; the image rows are padded to kRowPad >= 256)
    const int n_db_pad = (n_db + 255) / 256 * 256;
    int b1[kCT], b2[kCT];
#pragma unroll
    for (int t = 0; t < kCT; ++t) b1[t] = b2[t] = INT_MAX;

    // one 32-row database tile: A fragments (XOR-swizzled LDS image) and the
    // packed key bases of this lane's 16 rows (rows (j&3) + 8(j>>2) + 4h)
    auto load_frag = [&](const int8_t* A, const int32_t* N, int tile, v4i (&af)[4], v4i (&nt4)[4]) {
        const int r = tile + c;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
            af[s4] = *reinterpret_cast<const v4i*>(A + r * 128 + (((4 * h + s4) ^ (r & 7)) << 4));
#pragma unroll
        for (int q = 0; q < 4; ++q) nt4[q] = *reinterpret_cast<const v4i*>(N + tile + 4 * h + 8 * q);
    };
    auto mfma_tile = [&](const v4i (&af)[4], v16i (&acc)[kCT]) {
#pragma unroll
        for (int t = 0; t < kCT; ++t) {
            acc[t] = v16i{};
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4)
                acc[t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[s4], bq[t][s4], acc[t], 0, 0, 0);
        }
    };
    // epilogue of one tile for every column tile, pairs interleaved for ILP:
    // key = nt - 512*dot (v_mad_i32_i24; |dot| < 2^21 fits 24 bits; the
    // multiplier is a kernel argument so it is not strength-reduced).
    // Two keys x, y of one query per update; the two smallest of the
    // multiset {b1 <= b2, x, y} are
    //   b1' = min3(b1, x, y),  b2' = min(med3(b1, x, y), b2)
    // (b1 smallest: med3 = min(x, y); b1 in the middle: med3 = b1 <= b2;
    // b1 largest: med3 = max(x, y) <= b1 <= b2), so 3 VALU per 2
    // distances instead of med3 + min per distance.  Two consecutive
    // pairs share one b2 update, b2 = min3(b2, t_a, t_b) (the same
    // value as two min steps): 5 VALU per 4 distances.
    // Plain C min / max: the compiler selects v_min3_i32 / v_med3_i32 for
    // these shapes (checked in the ISA, tests/test_match_isa.py) and its
    // hazard recognizer sees every instruction.
    auto epilogue = [&](const v16i (&acc)[kCT], const v4i (&nt4)[4]) {
#pragma unroll
        for (int tp = 0; tp < kCT; tp += 2)
#pragma unroll
        for (int j = 0; j < 16; j += 4) {
            const int x0 = __mul24(acc[tp][j], a.kmul) + nt4[j >> 2][0];
            const int x1 = __mul24(acc[tp + 1][j], a.kmul) + nt4[j >> 2][0];
            const int y0 = __mul24(acc[tp][j + 1], a.kmul) + nt4[j >> 2][1];
            const int y1 = __mul24(acc[tp + 1][j + 1], a.kmul) + nt4[j >> 2][1];
            const int z0 = __mul24(acc[tp][j + 2], a.kmul) + nt4[j >> 2][2];
            const int z1 = __mul24(acc[tp + 1][j + 2], a.kmul) + nt4[j >> 2][2];
            const int w0 = __mul24(acc[tp][j + 3], a.kmul) + nt4[j >> 2][3];
            const int w1 = __mul24(acc[tp + 1][j + 3], a.kmul) + nt4[j >> 2][3];
            if (!kRatio) {
                b1[tp] = min3i(min3i(b1[tp], x0, y0), z0, w0);
                b1[tp + 1] = min3i(min3i(b1[tp + 1], x1, y1), z1, w1);
                continue;
            }
            // b1' through opaque(): no min(b1, x) shared with med3, so the
            // selector keeps v_min3 (a shared inner min is not one-use)
            const int ta0 = med3i(b1[tp], x0, y0), ta1 = med3i(b1[tp + 1], x1, y1);
            b1[tp] = min3i(b1[tp], opaque(x0), y0);
            b1[tp + 1] = min3i(b1[tp + 1], opaque(x1), y1);
            const int tb0 = med3i(b1[tp], z0, w0), tb1 = med3i(b1[tp + 1], z1, w1);
            b1[tp] = min3i(b1[tp], opaque(z0), w0);
            b1[tp + 1] = min3i(b1[tp + 1], opaque(z1), w1);
            b2[tp] = min3i(b2[tp], ta0, tb0);
            b2[tp + 1] = min3i(b2[tp + 1], ta1, tb1);
        }
    };
    // keys carry row & 255: the tile keys are merged into the running state
    // every 256 rows
    auto merge_window = [&](int base) {
#pragma unroll
        for (int t = 0; t < kCT; ++t) {
            merge_tile(g[t], b1[t], b2[t], base);
            b1[t] = INT_MAX; b2[t] = INT_MAX;
        }
    };

    // A stage is filled by all four waves' LDS DMA, and read by every wave:
    // each wave drains its own DMA (vmcnt) BEFORE the barrier.  __syncthreads
    // alone does not (gfx950's workgroup release fence does not wait for
    // loads), and the waitcnt pass places its LDS-DMA wait next to the first
    // aliasing ds_read, after the barrier, where it covers only the wave's
    // own part -- in the round-3 ISA it omitted it altogether on the stage
    // loop's back edge (the cause of the MUTUAL mismatch of the unrolled
    // build).
    auto stage_landed = [&] {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    };
    if (n_db_pad > 0) issue_to(sA0, sN0, 0);
    // one stage: its tiles from (A, N) while the next stage lands in (nA, nN)
    auto stage = [&](const int8_t* A, const int32_t* N, int8_t* nA, int32_t* nN, int sup) {
        stage_landed();    // this stage has landed in every wave's part; the other buffer is free
        if (sup + kStage < n_db_pad) issue_to(nA, nN, sup + kStage);
#pragma unroll MATCH_TILE_UNROLL
        for (int tile = 0; tile < kStage; tile += 32) {
            v4i af[4], nt4[4];
            load_frag(A, N, tile, af, nt4);
            v16i acc[kCT];
            mfma_tile(af, acc);
            epilogue(acc, nt4);
        }
        if (((sup + kStage) & 255) == 0) merge_window(sup + kStage - 256);
    };
    for (int sup = 0; sup < n_db_pad; sup += 2 * kStage) {
        stage(sA0, sN0, sA1, sN1, sup);
        if (sup + kStage < n_db_pad) stage(sA1, sN1, sA0, sN0, sup + kStage);
    }

#pragma unroll
    for (int t = 0; t < kCT; ++t) {
        merge_lanes(g[t]);
        const int q = qblk * kQB + wave * kQW + 32 * t + c;
        if (h == 0 && q < n_q) {
            const int nq = a.nrm[a.img_row0[q_img] + q];
            int idx = g[t].g1i, d1 = nq + g[t].g1v;
            if (kRatio) {
                const bool keep = n_db >= 2 && (float)d1 < a.r2 * (float)(nq + g[t].g2v);
                if (!keep) idx = -1;
            }
            if (n_db == 0) { idx = -1; d1 = -1; }
            a.out_idx[(int64_t)pair * a.out_stride + q] = idx;
            a.out_d[(int64_t)pair * a.out_stride + q] = idx >= 0 ? d1 : -1;
        }
    }
}

// MUTUAL: keep (q, t) iff nnJ[q] = t and nnI[t] = q.
__global__ void mutual_kernel(int32_t* __restrict__ idx_q, int32_t* __restrict__ d_q,
                              const int32_t* __restrict__ idx_t, const int32_t* __restrict__ pairs,
                              const int32_t* __restrict__ img_n, int n_pairs, int64_t stride) {
    const int pair = blockIdx.y;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (pair >= n_pairs) return;
    const int nI = img_n[pairs[2 * pair]];
    if (q >= nI) return;
    const int64_t o = (int64_t)pair * stride;
    const int t = idx_q[o + q];
    if (t < 0 || idx_t[o + t] != q) { idx_q[o + q] = -1; d_q[o + q] = -1; }
}

// ---- float descriptors that are not integers in [0, 255] -------------------
// (cv::Mat CV_32F behind LocalFrame/GlobalFrame::matchFeature, LocalFrame.h:38,
// Image.h:39-41).  OpenCV's SIFT stores saturate_cast<uchar> values in its
// float descriptors, so those take the exact u8 path above; anything else
// lands here: one query per thread, d = sum_k (q_k - a_k)^2 as an fmaf chain
// in k order (the oracle's restatement, bit for bit), database rows staged in
// LDS and read as broadcasts, first minimum (lowest index) wins as in top2().
struct MatchF32Args {
    const float* desc;         // padded rows x 128 (f32)
    const int64_t* img_row0;
    const int32_t* img_n;
    const int32_t* pairs;
    int32_t n_pairs;
    int32_t qblocks;           // 256-query blocks per pair
    int32_t swap;
    float r2;
    int64_t out_stride;
    int32_t* out_idx;
    int32_t* out_d;            // float bits of the squared distance
};

constexpr int kF32Rows = 64;   // database rows per LDS stage

template <bool kRatio>
__global__ __launch_bounds__(256) void match_f32_kernel(MatchF32Args a) {
    const int pair = blockIdx.x / a.qblocks, qblk = blockIdx.x - pair * a.qblocks;
    if (pair >= a.n_pairs) return;
    const int I = a.pairs[2 * pair], J = a.pairs[2 * pair + 1];
    const int db_img = a.swap ? J : I, q_img = a.swap ? I : J;
    const int n_db = a.img_n[db_img], n_q = a.img_n[q_img];
    if (qblk * 256 >= n_q) return;
    const int q = qblk * 256 + (int)threadIdx.x;
    const bool has_q = q < n_q;
    float qv[128];
    {
        const float4* src = reinterpret_cast<const float4*>(a.desc + (a.img_row0[q_img] + (has_q ? q : 0)) * 128);
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            const float4 v = src[k];
            qv[4 * k] = v.x; qv[4 * k + 1] = v.y; qv[4 * k + 2] = v.z; qv[4 * k + 3] = v.w;
        }
    }
    __shared__ __attribute__((aligned(16))) float sA[kF32Rows * 128];
    const float* db = a.desc + a.img_row0[db_img] * 128;
    float b1 = __builtin_inff(), b2 = __builtin_inff();
    int i1 = -1;
    for (int base = 0; base < n_db; base += kF32Rows) {
        const int nr = min(kF32Rows, n_db - base);
        __syncthreads();   // the previous stage is consumed
        for (int e = threadIdx.x; e < kF32Rows * 32; e += 256)
            reinterpret_cast<float4*>(sA)[e] =
                e < nr * 32 ? reinterpret_cast<const float4*>(db + (int64_t)base * 128)[e] : float4{0.f, 0.f, 0.f, 0.f};
        __syncthreads();
        for (int r = 0; r < nr; ++r) {
            const float4* row = reinterpret_cast<const float4*>(sA + r * 128);
            float d = 0.f;
#pragma unroll
            for (int k = 0; k < 32; ++k) {
                const float4 v = row[k];
                const float t0 = qv[4 * k] - v.x, t1 = qv[4 * k + 1] - v.y;
                const float t2 = qv[4 * k + 2] - v.z, t3 = qv[4 * k + 3] - v.w;
                d = __builtin_fmaf(t0, t0, d);
                d = __builtin_fmaf(t1, t1, d);
                d = __builtin_fmaf(t2, t2, d);
                d = __builtin_fmaf(t3, t3, d);
            }
            if (d < b1) {
                if (kRatio) b2 = b1;
                b1 = d;
                i1 = base + r;
            } else if (kRatio && d < b2) {
                b2 = d;
            }
        }
    }
    if (!has_q) return;
    int idx = i1;
    float d1 = b1;
    if (kRatio && !(n_db >= 2 && b1 < a.r2 * b2)) idx = -1;
    if (idx < 0) d1 = -1.f;
    a.out_idx[(int64_t)pair * a.out_stride + q] = idx;
    a.out_d[(int64_t)pair * a.out_stride + q] = __float_as_int(d1);
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// Order-independent digest: sum over pairs of mix(pair_id, sum over matches
// of mix(i, j, d)), plus the total match count.
__global__ void digest_kernel(const int32_t* __restrict__ idx, const int32_t* __restrict__ d,
                              const int32_t* __restrict__ pairs, const int32_t* __restrict__ img_n,
                              int mode, int64_t pair_base, int n_pairs, int64_t stride,
                              unsigned long long* out) {
    const int pair = blockIdx.x;
    if (pair >= n_pairs) return;
    const int I = pairs[2 * pair], J = pairs[2 * pair + 1];
    const bool qJ = mode != SFM_MATCH_MUTUAL;   // outputs per query of J
    const int n_out = qJ ? img_n[J] : img_n[I];
    uint64_t h = 0, cnt = 0;
    for (int q = threadIdx.x; q < n_out; q += blockDim.x) {
        const int m = idx[(int64_t)pair * stride + q];
        if (m < 0) continue;
        const uint32_t ii = qJ ? (uint32_t)m : (uint32_t)q;
        const uint32_t jj = qJ ? (uint32_t)q : (uint32_t)m;
        h += mix64(((uint64_t)ii << 32 | jj) ^ ((uint64_t)(uint32_t)d[(int64_t)pair * stride + q] << 21));
        ++cnt;
    }
    __shared__ unsigned long long sh[2][256];
    sh[0][threadIdx.x] = h;
    sh[1][threadIdx.x] = cnt;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) { sh[0][threadIdx.x] += sh[0][threadIdx.x + o]; sh[1][threadIdx.x] += sh[1][threadIdx.x + o]; }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        atomicAdd(&out[0], (unsigned long long)mix64(sh[0][0] + 0x9E3779B97F4A7C15ULL * (uint64_t)(pair_base + pair + 1)));
        atomicAdd(&out[1], sh[1][0]);
    }
}

}  // namespace
}  // namespace sfm

using namespace sfm;

struct sfm_match_plan {
    sfm_ctx* ctx = nullptr;
    int32_t n_img = 0;
    std::vector<int64_t> row0;   // padded row start per image
    std::vector<int32_t> nrows;
    int32_t max_n = 0;
    int64_t rows = 0;            // padded rows in total
    DBuf<uint8_t> desc;
    DBuf<float> descf;           // f32 collection that is not integer-valued (match_f32_kernel)
    bool f32 = false;
    DBuf<int32_t> nrm, ntr, img_n;
    DBuf<int64_t> img_row0;
    // last run
    int32_t mode = 0;
    int64_t n_pairs = 0, stride = 0;
    std::vector<int32_t> pairs_h;
    DBuf<int32_t> pairs_d, out_idx, out_d, tmp_idx, tmp_d;
    DBuf<unsigned long long> digest;
    // cascade hashing tables, built by the first CASCADE run and rebuilt when
    // the set of images in the pair list (the zero-mean input) changes
    std::vector<int32_t> casc_used;
    bool casc_ready = false;
    bool casc_pinned = false;    // set by sfm_match_plan_cascade_index
    DBuf<float> casc_proj, casc_zm;
    DBuf<int64_t> casc_colsum;
    DBuf<uint32_t> casc_code;
    DBuf<uint64_t> casc_bkt;
    DBuf<int32_t> casc_boff, casc_blist, casc_img;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0;
    int64_t launches = 0;
};

namespace {

// srcs (optional): image i's rows start at srcs[i] instead of desc + 128 off[i]
void upload_collection(sfm_match_plan* p, const uint8_t* desc, const int64_t* off, int32_t n_img,
                       const uint8_t* const* srcs = nullptr) {
    hipStream_t s = p->ctx->stream;
    p->n_img = n_img;
    p->row0.resize(n_img);
    p->nrows.resize(n_img);
    int64_t rows = 0;
    for (int i = 0; i < n_img; ++i) {
        const int64_t n = off[i + 1] - off[i];
        SFM_REQUIRE(n >= 0 && n < (1 << 24), SFM_ERR_INVALID_ARG, "image %d has %lld rows", i,
                    (long long)n);
        p->row0[i] = rows;
        p->nrows[i] = (int32_t)n;
        p->max_n = std::max<int32_t>(p->max_n, (int32_t)n);
        rows += (n + kRowPad - 1) / kRowPad * kRowPad;
    }
    rows += kRowPad;  // guard rows for tile over-reads
    p->rows = rows;
    PhaseTimer tm("upload_collection");
    if (PhaseTimer::on()) {   // diagnostic: is anything still queued before this call?
        SFM_HIP(hipStreamSynchronize(s));
        tm.mark("presync");
    }
    // page-locked staging from the context's host cache (a pageable source
    // made each upload of a 300-image loop's collection cost milliseconds)
    HostVec<uint8_t> staging((size_t)rows * 128, 128);  // pad rows -> a' = 0
    HostVec<int64_t> rstart(rows, 0);
    HostVec<int32_t> rvalid(rows, 0);
    for (int i = 0; i < n_img; ++i) {
        if (p->nrows[i])
            std::memcpy(&staging[(size_t)p->row0[i] * 128], srcs ? srcs[i] : desc + off[i] * 128,
                        (size_t)p->nrows[i] * 128);
        const int64_t padded = (p->nrows[i] + kRowPad - 1) / kRowPad * kRowPad;
        for (int64_t r = 0; r < padded; ++r) {
            rstart[p->row0[i] + r] = p->row0[i];
            rvalid[p->row0[i] + r] = r < p->nrows[i];
        }
    }
    tm.mark("stage");
    p->desc.alloc(staging.size());
    tm.mark("alloc");
    p->desc.upload(staging.data(), staging.size(), s);
    if (PhaseTimer::on()) SFM_HIP(hipStreamSynchronize(s));
    tm.mark("copy");
    DBuf<int64_t> rs;
    DBuf<int32_t> rv;
    rs.alloc(rows);
    rv.alloc(rows);
    rs.upload(rstart.data(), rows, s);
    rv.upload(rvalid.data(), rows, s);
    p->nrm.alloc(rows);
    p->ntr.alloc(rows);
    hipLaunchKernelGGL(prep_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, p->desc.p,
                       p->nrm.p, p->ntr.p, rs.p, rv.p, rows);
    SFM_HIP(hipGetLastError());
    p->img_n.alloc(n_img);
    p->img_n.upload(p->nrows.data(), n_img, s);
    p->img_row0.alloc(n_img);
    p->img_row0.upload(p->row0.data(), n_img, s);
    tm.mark("rest");
    SFM_HIP(hipStreamSynchronize(s));  // staging buffers die here
    tm.mark("sync");
}

// float descriptors: integers in [0, 255] (what cv::SIFT stores) are
// converted exactly and take the u8 path; anything else is kept as f32
bool f32_is_u8(const float* d, int64_t n) {
    for (int64_t k = 0; k < n; ++k) {
        const float v = d[k];
        if (!(v >= 0.f && v <= 255.f) || v != (float)(int)v) return false;
    }
    return true;
}

void upload_collection_f32(sfm_match_plan* p, const float* desc, const int64_t* off, int32_t n_img,
                           const float* const* srcs = nullptr) {
    bool u8 = true;
    for (int i = 0; i < n_img && u8; ++i)
        u8 = f32_is_u8(srcs ? srcs[i] : desc + off[i] * 128, (off[i + 1] - off[i]) * 128);
    if (u8) {
        std::vector<uint8_t> b((size_t)std::max<int64_t>(off[n_img] - off[0], 0) * 128);
        for (int i = 0; i < n_img; ++i) {
            const float* src = srcs ? srcs[i] : desc + off[i] * 128;
            uint8_t* dst = b.data() + (off[i] - off[0]) * 128;
            for (int64_t k = 0; k < (off[i + 1] - off[i]) * 128; ++k) dst[k] = (uint8_t)src[k];
        }
        std::vector<int64_t> o(off, off + n_img + 1);
        for (auto& v : o) v -= off[0];
        upload_collection(p, b.data(), o.data(), n_img);
        return;
    }
    hipStream_t s = p->ctx->stream;
    p->f32 = true;
    p->n_img = n_img;
    p->row0.resize(n_img);
    p->nrows.resize(n_img);
    int64_t rows = 0;
    for (int i = 0; i < n_img; ++i) {
        const int64_t n = off[i + 1] - off[i];
        SFM_REQUIRE(n >= 0 && n < (1 << 24), SFM_ERR_INVALID_ARG, "image %d has %lld rows", i, (long long)n);
        p->row0[i] = rows;
        p->nrows[i] = (int32_t)n;
        p->max_n = std::max<int32_t>(p->max_n, (int32_t)n);
        rows += (n + kRowPad - 1) / kRowPad * kRowPad;
    }
    rows += kRowPad;
    p->rows = rows;
    HostVec<float> staging((size_t)rows * 128, 0.f);
    for (int i = 0; i < n_img; ++i)
        if (p->nrows[i])
            std::memcpy(&staging[(size_t)p->row0[i] * 128], srcs ? srcs[i] : desc + off[i] * 128,
                        (size_t)p->nrows[i] * 128 * sizeof(float));
    p->descf.alloc(staging.size());
    p->descf.upload(staging.data(), staging.size(), s);
    p->img_n.alloc(n_img);
    p->img_n.upload(p->nrows.data(), n_img, s);
    p->img_row0.alloc(n_img);
    p->img_row0.upload(p->row0.data(), n_img, s);
    SFM_HIP(hipStreamSynchronize(s));  // staging dies here
}

CascTables casc_tables(sfm_match_plan* p) {
    CascTables t;
    t.desc = reinterpret_cast<const int8_t*>(p->desc.p);
    t.nrm = p->nrm.p;
    t.img_row0 = p->img_row0.p;
    t.img_n = p->img_n.p;
    t.rows = p->rows;
    t.code = p->casc_code.p;
    t.bkt = p->casc_bkt.p;
    t.boff = p->casc_boff.p;
    t.blist = p->casc_blist.p;
    return t;
}

// Run the top-2 kernel over pairs [0, n_pairs) in launch batches.
void run_top2(sfm_match_plan* p, const int32_t* pairs_d, int64_t n_pairs, int swap, int ratio_test,
              float r2, int32_t* out_idx, int32_t* out_d, int64_t stride) {
    hipStream_t s = p->ctx->stream;
    if (p->f32) {
        const int qblocks = std::max(1, (p->max_n + 255) / 256);
        const int64_t batch = std::max<int64_t>(1, ((int64_t)1 << 22) / qblocks);
        for (int64_t b0 = 0; b0 < n_pairs; b0 += batch) {
            const int64_t nb = std::min(batch, n_pairs - b0);
            MatchF32Args a;
            a.desc = p->descf.p;
            a.img_row0 = p->img_row0.p;
            a.img_n = p->img_n.p;
            a.pairs = pairs_d + 2 * b0;
            a.n_pairs = (int32_t)nb;
            a.qblocks = qblocks;
            a.swap = swap;
            a.r2 = r2;
            a.out_stride = stride;
            a.out_idx = out_idx + b0 * stride;
            a.out_d = out_d + b0 * stride;
            if (ratio_test)
                hipLaunchKernelGGL(match_f32_kernel<true>, dim3((unsigned)(nb * qblocks)), dim3(256), 0, s, a);
            else
                hipLaunchKernelGGL(match_f32_kernel<false>, dim3((unsigned)(nb * qblocks)), dim3(256), 0, s, a);
            SFM_HIP(hipGetLastError());
            ++p->launches;
        }
        return;
    }
    const int qblocks = std::max(1, (p->max_n + kQB - 1) / kQB);
    const int64_t max_wg = 1 << 22;
    const int64_t batch = std::max<int64_t>(1, max_wg / qblocks);
    for (int64_t b0 = 0; b0 < n_pairs; b0 += batch) {
        const int64_t nb = std::min(batch, n_pairs - b0);
        MatchArgs a;
        a.desc = reinterpret_cast<const int8_t*>(p->desc.p);
        a.nrm = p->nrm.p;
        a.ntr = p->ntr.p;
        a.img_row0 = p->img_row0.p;
        a.img_n = p->img_n.p;
        a.pairs = pairs_d + 2 * b0;
        a.n_pairs = (int32_t)nb;
        a.qblocks = qblocks;
        a.swap = swap;
        a.ratio_test = ratio_test;
        a.kmul = -512;
        a.r2 = r2;
        a.out_stride = stride;
        a.out_idx = out_idx + b0 * stride;
        a.out_d = out_d + b0 * stride;
        if (ratio_test)
            hipLaunchKernelGGL(match_top2_kernel<true>, dim3((unsigned)(nb * qblocks)), dim3(kThreads), 0, s, a);
        else
            hipLaunchKernelGGL(match_top2_kernel<false>, dim3((unsigned)(nb * qblocks)), dim3(kThreads), 0, s, a);
        SFM_HIP(hipGetLastError());
        ++p->launches;
    }
}

// Hash tables for the images of this pair list (zero-mean over exactly those
// images, as Cascade_Hashing_Matcher_Regions' used_index).
void casc_prepare(sfm_match_plan* p, const int32_t* pairs, int64_t n_pairs, bool pin) {
    hipStream_t s = p->ctx->stream;
    std::vector<char> seen(p->n_img, 0);
    for (int64_t q = 0; q < 2 * n_pairs; ++q) seen[pairs[q]] = 1;
    std::vector<int32_t> used;
    for (int i = 0; i < p->n_img; ++i)
        if (seen[i]) used.push_back(i);
    if (p->casc_ready) {
        if (used == p->casc_used) {
            p->casc_pinned = p->casc_pinned || pin;
            return;
        }
        if (!pin && p->casc_pinned &&
            std::includes(p->casc_used.begin(), p->casc_used.end(), used.begin(), used.end()))
            return;   // a part of the indexed list
    }
    p->casc_pinned = pin;
    SFM_REQUIRE(p->max_n < (1 << 21), SFM_ERR_UNSUPPORTED,
                "cascade hashing: %d descriptors in one image (limit 2^21)", p->max_n);
    CascTables t = casc_tables(p);
    if (!p->casc_proj.p) {
        std::vector<float> proj;
        casc_projections(proj);
        p->casc_proj.alloc(proj.size());
        p->casc_proj.upload(proj.data(), proj.size(), s);
        p->casc_zm.alloc(kCascCode);
        p->casc_colsum.alloc((size_t)std::max(1, p->n_img) * kCascCode);
        p->casc_code.alloc((size_t)p->rows * 4);
        p->casc_bkt.alloc((size_t)p->rows);
        p->casc_boff.alloc((size_t)std::max(1, p->n_img) * kCascGroups * (kCascBuckets + 1));
        p->casc_blist.alloc((size_t)p->rows * kCascGroups);
        p->casc_img.alloc(std::max(1, p->n_img));
        t = casc_tables(p);
        casc_colsum(t, p->n_img, p->casc_colsum.p, s);
    }
    std::vector<int64_t> colsum((size_t)p->n_img * kCascCode);
    if (p->n_img)
        SFM_HIP(hipMemcpyAsync(colsum.data(), p->casc_colsum.p, colsum.size() * 8,
                               hipMemcpyDeviceToHost, s));
    SFM_HIP(hipStreamSynchronize(s));
    float zm[kCascCode];
    casc_zero_mean(colsum.data(), p->nrows.data(), used, zm);
    p->casc_zm.upload(zm, kCascCode, s);
    if (!used.empty()) p->casc_img.upload(used.data(), used.size(), s);
    casc_hash(t, p->casc_proj.p, p->casc_zm.p, p->casc_img.p, (int)used.size(), p->max_n, s);
    SFM_HIP(hipStreamSynchronize(s));   // host zm / image list die here
    p->casc_used = std::move(used);
    p->casc_ready = true;
}

void run_cascade(sfm_match_plan* p, int64_t n_pairs, float r2) {
    const int qblocks = std::max(1, (p->max_n + kCascQB - 1) / kCascQB);
    const int64_t batch = std::max<int64_t>(1, (int64_t)(1 << 22) / qblocks);
    for (int64_t b0 = 0; b0 < n_pairs; b0 += batch) {
        const int64_t nb = std::min(batch, n_pairs - b0);
        CascMatchArgs a;
        a.t = casc_tables(p);
        a.pairs = p->pairs_d.p + 2 * b0;
        a.n_pairs = (int32_t)nb;
        a.qblocks = qblocks;
        a.r2 = r2;
        a.out_stride = p->stride;
        a.out_idx = p->out_idx.p + b0 * p->stride;
        a.out_d = p->out_d.p + b0 * p->stride;
        casc_match(a, p->max_n, p->ctx->stream);
        ++p->launches;
    }
}

void run_pairs(sfm_match_plan* p, const int32_t* pairs, int64_t n_pairs, const sfm_match_options* o,
               bool timed = true) {
    hipStream_t s = p->ctx->stream;
    SFM_REQUIRE(o && (o->mode == SFM_MATCH_RATIO || o->mode == SFM_MATCH_MUTUAL ||
                      o->mode == SFM_MATCH_CASCADE),
                SFM_ERR_INVALID_ARG, "bad match options");
    for (int64_t q = 0; q < n_pairs; ++q)
        SFM_REQUIRE(pairs[2 * q] >= 0 && pairs[2 * q] < p->n_img && pairs[2 * q + 1] >= 0 &&
                        pairs[2 * q + 1] < p->n_img,
                    SFM_ERR_INVALID_ARG, "pair %lld out of range", (long long)q);
    SFM_REQUIRE(!(p->f32 && o->mode == SFM_MATCH_CASCADE), SFM_ERR_UNSUPPORTED,
                "cascade hashing needs integer descriptors in [0, 255] (this f32 collection is not)");
    if (o->mode == SFM_MATCH_CASCADE) casc_prepare(p, pairs, n_pairs, false);
    p->mode = o->mode;
    p->n_pairs = n_pairs;
    p->stride = std::max<int64_t>(1, p->max_n);
    p->pairs_h.assign(pairs, pairs + 2 * n_pairs);
    if ((int64_t)p->pairs_d.n < 2 * n_pairs) p->pairs_d.alloc(std::max<int64_t>(2, 2 * n_pairs));
    p->pairs_d.upload(pairs, 2 * n_pairs, s);
    const size_t need = (size_t)std::max<int64_t>(1, n_pairs * p->stride);
    if (p->out_idx.n < need) { p->out_idx.alloc(need); p->out_d.alloc(need); }
    p->launches = 0;
    if (timed && !p->ev0) { SFM_HIP(hipEventCreate(&p->ev0)); SFM_HIP(hipEventCreate(&p->ev1)); }
    if (timed) SFM_HIP(hipEventRecord(p->ev0, s));
    if (n_pairs > 0) {
        if (o->mode == SFM_MATCH_CASCADE) {
            run_cascade(p, n_pairs, o->ratio * o->ratio);
        } else if (o->mode == SFM_MATCH_RATIO) {
            run_top2(p, p->pairs_d.p, n_pairs, 0, 1, o->ratio * o->ratio, p->out_idx.p, p->out_d.p,
                     p->stride);
        } else {
            if (p->tmp_idx.n < need) { p->tmp_idx.alloc(need); p->tmp_d.alloc(need); }
            // nn over J for every row of I, and nn over I for every row of J
            run_top2(p, p->pairs_d.p, n_pairs, 1, 0, 0.f, p->out_idx.p, p->out_d.p, p->stride);
            run_top2(p, p->pairs_d.p, n_pairs, 0, 0, 0.f, p->tmp_idx.p, p->tmp_d.p, p->stride);
            dim3 grid((unsigned)((p->max_n + 255) / 256), 1, 1);
            for (int64_t b0 = 0; b0 < n_pairs; b0 += 65535) {
                const int64_t nb = std::min<int64_t>(65535, n_pairs - b0);
                grid.y = (unsigned)nb;
                hipLaunchKernelGGL(mutual_kernel, grid, dim3(256), 0, s, p->out_idx.p + b0 * p->stride,
                                   p->out_d.p + b0 * p->stride, p->tmp_idx.p + b0 * p->stride,
                                   p->pairs_d.p + 2 * b0, p->img_n.p, (int)nb, p->stride);
                SFM_HIP(hipGetLastError());
                ++p->launches;
            }
        }
    }
    if (timed) SFM_HIP(hipEventRecord(p->ev1, s));
}

}  // namespace

extern "C" int sfm_match_plan_create(sfm_ctx* ctx, const uint8_t* desc, const int64_t* offsets,
                                     int32_t n_img, sfm_match_plan** out) {
    return guarded([&] {
        SFM_REQUIRE(ctx && out && offsets && n_img >= 0, SFM_ERR_INVALID_ARG, "null argument");
        SFM_REQUIRE(desc || offsets[n_img] == 0, SFM_ERR_INVALID_ARG, "null descriptors");
        CtxScope scope_(ctx);
        auto* p = new sfm_match_plan;
        p->ctx = ctx;
        try {
            upload_collection(p, desc, offsets, n_img);
        } catch (...) {
            delete p;
            throw;
        }
        *out = p;
        return SFM_OK;
    });
}

extern "C" int sfm_match_plan_run(sfm_match_plan* p, const int32_t* pairs, int64_t n_pairs,
                                  const sfm_match_options* o, int64_t* total) {
    return guarded([&] {
        SFM_REQUIRE(p && (pairs || n_pairs == 0) && n_pairs >= 0, SFM_ERR_INVALID_ARG,
                    "bad arguments");
        CtxScope scope_(p->ctx);
        run_pairs(p, pairs, n_pairs, o);
        if (total) {
            uint64_t dg;
            (void)dg;
            if (!p->digest.p) p->digest.alloc(2);
            p->digest.zero(p->ctx->stream);
            for (int64_t b0 = 0; b0 < n_pairs; b0 += 65535) {
                const int64_t nb = std::min<int64_t>(65535, n_pairs - b0);
                hipLaunchKernelGGL(digest_kernel, dim3((unsigned)nb), dim3(256), 0, p->ctx->stream,
                                   p->out_idx.p + b0 * p->stride, p->out_d.p + b0 * p->stride,
                                   p->pairs_d.p + 2 * b0, p->img_n.p, p->mode, b0, (int)nb,
                                   p->stride, p->digest.p);
                SFM_HIP(hipGetLastError());
            }
            unsigned long long h[2];
            SFM_HIP(hipMemcpyAsync(h, p->digest.p, sizeof h, hipMemcpyDeviceToHost, p->ctx->stream));
            SFM_HIP(hipStreamSynchronize(p->ctx->stream));
            *total = (int64_t)h[1];
        }
        return SFM_OK;
    });
}

extern "C" int sfm_match_plan_cascade_index(sfm_match_plan* p, const int32_t* pairs, int64_t n_pairs) {
    return guarded([&] {
        SFM_REQUIRE(p && (pairs || n_pairs == 0) && n_pairs >= 0, SFM_ERR_INVALID_ARG,
                    "bad arguments");
        for (int64_t q = 0; q < 2 * n_pairs; ++q)
            SFM_REQUIRE(pairs[q] >= 0 && pairs[q] < p->n_img, SFM_ERR_INVALID_ARG,
                        "pair %lld out of range", (long long)(q / 2));
        SFM_REQUIRE(!p->f32, SFM_ERR_UNSUPPORTED,
                    "cascade hashing needs integer descriptors in [0, 255] (this f32 collection is not)");
        CtxScope scope_(p->ctx);
        casc_prepare(p, pairs, n_pairs, true);
        return SFM_OK;
    });
}

extern "C" int sfm_match_plan_digest(sfm_match_plan* p, uint64_t* digest) {
    return guarded([&] {
        SFM_REQUIRE(p && digest, SFM_ERR_INVALID_ARG, "null argument");
        CtxScope scope_(p->ctx);
        if (!p->digest.p) p->digest.alloc(2);
        p->digest.zero(p->ctx->stream);
        for (int64_t b0 = 0; b0 < p->n_pairs; b0 += 65535) {
            const int64_t nb = std::min<int64_t>(65535, p->n_pairs - b0);
            hipLaunchKernelGGL(digest_kernel, dim3((unsigned)nb), dim3(256), 0, p->ctx->stream,
                               p->out_idx.p + b0 * p->stride, p->out_d.p + b0 * p->stride,
                               p->pairs_d.p + 2 * b0, p->img_n.p, p->mode, b0, (int)nb, p->stride,
                               p->digest.p);
            SFM_HIP(hipGetLastError());
        }
        unsigned long long h[2];
        SFM_HIP(hipMemcpyAsync(h, p->digest.p, sizeof h, hipMemcpyDeviceToHost, p->ctx->stream));
        SFM_HIP(hipStreamSynchronize(p->ctx->stream));
        *digest = h[0];
        return SFM_OK;
    });
}

namespace {
// D = int32_t: exact integer squared distances (u8 collections); D = float:
// float squared distances (any collection; integers convert exactly)
template <class D>
void fetch_results(sfm_match_plan* p, int64_t* counts, uint32_t* i, uint32_t* j, D* d2) {
    const size_t n = (size_t)(p->n_pairs * p->stride);
    std::vector<int32_t> hi(n), hd(n);
    if (n) {
        SFM_HIP(hipMemcpyAsync(hi.data(), p->out_idx.p, n * 4, hipMemcpyDeviceToHost, p->ctx->stream));
        SFM_HIP(hipMemcpyAsync(hd.data(), p->out_d.p, n * 4, hipMemcpyDeviceToHost, p->ctx->stream));
    }
    SFM_HIP(hipStreamSynchronize(p->ctx->stream));
    int64_t off = 0;
    std::vector<std::pair<uint64_t, int32_t>> v;
    for (int64_t q = 0; q < p->n_pairs; ++q) {
        const int I = p->pairs_h[2 * q], J = p->pairs_h[2 * q + 1];
        const bool qJ = p->mode != SFM_MATCH_MUTUAL;
        const int n_out = qJ ? p->nrows[J] : p->nrows[I];
        v.clear();
        for (int t = 0; t < n_out; ++t) {
            const int m = hi[(size_t)q * p->stride + t];
            if (m < 0) continue;
            const uint32_t ii = qJ ? (uint32_t)m : (uint32_t)t;
            const uint32_t jj = qJ ? (uint32_t)t : (uint32_t)m;
            v.emplace_back(((uint64_t)ii << 32) | jj, hd[(size_t)q * p->stride + t]);
        }
        std::sort(v.begin(), v.end());  // IndMatch::getDeduplicated order
        counts[q] = (int64_t)v.size();
        if (i) {
            for (const auto& m : v) {
                i[off] = (uint32_t)(m.first >> 32);
                j[off] = (uint32_t)(m.first & 0xffffffffu);
                if constexpr (std::is_same<D, float>::value) {
                    float f;
                    if (p->f32) std::memcpy(&f, &m.second, 4);
                    else f = (float)m.second;
                    d2[off] = f;
                } else {
                    d2[off] = m.second;
                }
                ++off;
            }
        }
    }
}
}  // namespace

extern "C" int sfm_match_plan_fetch(sfm_match_plan* p, int64_t* counts, uint32_t* i, uint32_t* j,
                                    int32_t* d2) {
    return guarded([&] {
        SFM_REQUIRE(p && counts, SFM_ERR_INVALID_ARG, "null argument");
        SFM_REQUIRE(!p->f32, SFM_ERR_INVALID_ARG,
                    "float distances: this collection is not integer-valued (sfm_match_plan_fetch_f32)");
        CtxScope scope_(p->ctx);
        fetch_results(p, counts, i, j, d2);
        return SFM_OK;
    });
}

extern "C" int sfm_match_plan_fetch_f32(sfm_match_plan* p, int64_t* counts, uint32_t* i, uint32_t* j,
                                        float* d2) {
    return guarded([&] {
        SFM_REQUIRE(p && counts, SFM_ERR_INVALID_ARG, "null argument");
        CtxScope scope_(p->ctx);
        fetch_results(p, counts, i, j, d2);
        return SFM_OK;
    });
}

extern "C" int sfm_match_plan_create_f32(sfm_ctx* ctx, const float* desc, const int64_t* offsets,
                                         int32_t n_img, sfm_match_plan** out) {
    return guarded([&] {
        SFM_REQUIRE(ctx && out && offsets && n_img >= 0, SFM_ERR_INVALID_ARG, "null argument");
        SFM_REQUIRE(desc || offsets[n_img] == offsets[0], SFM_ERR_INVALID_ARG, "null descriptors");
        CtxScope scope_(ctx);
        auto* p = new sfm_match_plan;
        p->ctx = ctx;
        try {
            upload_collection_f32(p, desc, offsets, n_img);
        } catch (...) {
            delete p;
            throw;
        }
        *out = p;
        return SFM_OK;
    });
}

extern "C" int sfm_match_plan_get_last_ms(sfm_match_plan* p, double* ms, int64_t* launches) {
    return guarded([&] {
        SFM_REQUIRE(p && ms, SFM_ERR_INVALID_ARG, "null argument");
        float f = 0.f;
        if (p->ev0) {
            SFM_HIP(hipEventSynchronize(p->ev1));
            SFM_HIP(hipEventElapsedTime(&f, p->ev0, p->ev1));
        }
        *ms = f;
        if (launches) *launches = p->launches;
        return SFM_OK;
    });
}

extern "C" int sfm_match_plan_destroy(sfm_match_plan* p) {
    return guarded([&] {
        if (!p) return SFM_OK;
        CtxScope scope_(p->ctx);
        (void)hipStreamSynchronize(p->ctx->stream);
        if (p->ev0) { (void)hipEventDestroy(p->ev0); (void)hipEventDestroy(p->ev1); }
        delete p;
        return SFM_OK;
    });
}

extern "C" int sfm_match_dense(sfm_ctx* ctx, const uint8_t* a, int32_t n_a, const uint8_t* b,
                               int32_t n_b, const sfm_match_options* o, int32_t* match_idx,
                               int32_t* match_d2) {
    return guarded([&] {
        SFM_REQUIRE(ctx && o && match_idx && match_d2 && n_a >= 0 && n_b >= 0 &&
                        (a || n_a == 0) && (b || n_b == 0),
                    SFM_ERR_INVALID_ARG, "bad arguments");
        CtxScope scope_(ctx);
        PhaseTimer tm("sfm_match_dense");
        const int64_t off[3] = {0, n_a, (int64_t)n_a + n_b};
        const uint8_t* srcs[2] = {a, b};
        sfm_match_plan plan;
        plan.ctx = ctx;
        tm.mark("stage");
        upload_collection(&plan, nullptr, off, 2, srcs);
        tm.mark("upload");
        const int32_t pair[2] = {0, 1};
        run_pairs(&plan, pair, 1, o, false);
        tm.mark("launch");
        const int32_t n_out = o->mode != SFM_MATCH_MUTUAL ? n_b : n_a;
        if (n_out) {
            SFM_HIP(hipMemcpyAsync(match_idx, plan.out_idx.p, (size_t)n_out * 4, hipMemcpyDeviceToHost, ctx->stream));
            SFM_HIP(hipMemcpyAsync(match_d2, plan.out_d.p, (size_t)n_out * 4, hipMemcpyDeviceToHost, ctx->stream));
        }
        SFM_HIP(hipStreamSynchronize(ctx->stream));
        tm.mark("sync+download");
        return SFM_OK;
    });
}

extern "C" int sfm_match_dense_f32(sfm_ctx* ctx, const float* a, int32_t n_a, const float* b, int32_t n_b,
                                   const sfm_match_options* o, int32_t* match_idx, float* match_d2) {
    return guarded([&] {
        SFM_REQUIRE(ctx && o && match_idx && match_d2 && n_a >= 0 && n_b >= 0 && (a || n_a == 0) &&
                        (b || n_b == 0),
                    SFM_ERR_INVALID_ARG, "bad arguments");
        CtxScope scope_(ctx);
        const int64_t off[3] = {0, n_a, (int64_t)n_a + n_b};
        const float* srcs[2] = {a, b};
        sfm_match_plan plan;
        plan.ctx = ctx;
        upload_collection_f32(&plan, nullptr, off, 2, srcs);
        const int32_t pair[2] = {0, 1};
        run_pairs(&plan, pair, 1, o, false);
        const int32_t n_out = o->mode != SFM_MATCH_MUTUAL ? n_b : n_a;
        std::vector<int32_t> d(std::max(n_out, 1));
        if (n_out) {
            SFM_HIP(hipMemcpyAsync(match_idx, plan.out_idx.p, (size_t)n_out * 4, hipMemcpyDeviceToHost, ctx->stream));
            SFM_HIP(hipMemcpyAsync(d.data(), plan.out_d.p, (size_t)n_out * 4, hipMemcpyDeviceToHost, ctx->stream));
        }
        SFM_HIP(hipStreamSynchronize(ctx->stream));
        for (int32_t q = 0; q < n_out; ++q) {
            if (match_idx[q] < 0) { match_d2[q] = -1.f; continue; }
            if (plan.f32) std::memcpy(&match_d2[q], &d[q], 4);
            else match_d2[q] = (float)d[q];
        }
        return SFM_OK;
    });
}
