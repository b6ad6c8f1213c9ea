// Cascade-hashing descriptor matching on CDNA4 (gfx950): the live default
// matcher of the reference, OpenMVG Cascade_Hashing_Matcher_Regions(0.8)
// selected by "AUTO" (src/sparseBuilder/sparseBuilder.cpp:811-814,911-914).
//
// Algorithm (OpenMVG cascade_hasher.hpp, after Cheng et al. 2014; restated
// in oracle/cascade_oracle.cpp, which is the bit-exact spec of this file):
//   * every descriptor x (uint8 -> float, minus the collection's zero-mean
//     descriptor) gets a 128-bit code sign(P x) and 6 bucket ids of 10 bits,
//     sign(S_g x) MSB first, from fixed Gaussian projections;
//   * a query q of image J collects the descriptors of image I sharing one of
//     its 6 buckets (first occurrence wins), orders them by Hamming distance
//     of the codes (stable), re-ranks the first 10 by exact L2^2 and keeps
//     the best if d1 < fl32(ratio^2) * d2; fewer than 3 collected candidates
//     or fewer than 2 distinct ones give no match.
// The projections are fp32 dot products with a fixed fma order (k = 0..127),
// so the hash bits are reproducible on the CPU; distances are exact integers.
//
// Kernels:
//   casc_colsum_kernel  per image column sums (zero-mean input), HBM-bound.
//   casc_hash_mfma_kernel  the 188 projections of 16 descriptors per wave as a
//                       [16 x 128] x [128 x 192] product on v_mfma_f32_16x16x4_f32
//                       (exact k-ordered fmaf chain), signs gathered by ballot.
//   casc_bucket_kernel  one wave per (image, group): LDS histogram, scan and
//                       a stable ballot-ranked scatter (lists stay ascending).
//   casc_match_kernel   one thread per query; candidates of image I are read
//                       from L2 (blockIdx is XCD-aware so one pair's query
//                       blocks share an XCD); re-rank with v_dot4_i32_i8.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <random>
#include <utility>

#include "cascade.h"
#include "common.h"

namespace sfm {

void casc_projections(std::vector<float>& proj) {
    // CascadeHasher::Init(gen, 128): d(gen) for primary(i, j), i-major, then
    // secondary[g](k, j) for g, k, j.
    std::mt19937 gen(std::mt19937::default_seed);
    std::normal_distribution<> d(0, 1);
    proj.assign((size_t)kCascProjRows * kCascCode, 0.f);
    for (int r = 0; r < kCascProjRows; ++r)
        for (int j = 0; j < kCascCode; ++j) proj[(size_t)r * kCascCode + j] = (float)d(gen);
}

void casc_zero_mean(const int64_t* colsum, const int32_t* img_n, const std::vector<int32_t>& used,
                    float* zm) {
    // GetZeroMeanDescriptor(per-image matrix) = float column sums / float(n)
    // (sums of <= 2^16 uint8 values are exact in float); then the mean of the
    // per-image means (empty images contribute zero rows), accumulated here
    // in double in ascending image order.
    for (int c = 0; c < kCascCode; ++c) {
        double acc = 0.0;
        for (const int32_t I : used) {
            const int32_t n = img_n[I];
            if (n > 0) acc += (double)((float)colsum[(int64_t)I * kCascCode + c] / (float)n);
        }
        zm[c] = used.empty() ? 0.f : (float)(acc / (double)used.size());
    }
}

namespace {

__global__ __launch_bounds__(128) void casc_colsum_kernel(const int8_t* __restrict__ desc,
                                                          const int64_t* __restrict__ img_row0,
                                                          const int32_t* __restrict__ img_n,
                                                          int64_t* __restrict__ colsum) {
    const int I = blockIdx.x, c = threadIdx.x;
    const int8_t* d = desc + img_row0[I] * 128 + c;
    const int n = img_n[I];
    int64_t s = 0;
    for (int r = 0; r < n; ++r) s += (int)d[(int64_t)r * 128] + 128;
    colsum[(int64_t)I * 128 + c] = s;
}


template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// Projections on the f32 MFMA (v_mfma_f32_16x16x4_f32): the result
// of one instruction is the k-ordered fmaf chain fma(a3,b3, .. fma(a0,b0,C)),
// and chaining the 32 k-steps in k order reproduces the sequential
// k = 0..127 fmaf chain of the oracle bit for bit.
//   A = 16 descriptors x 4 k (lane l: descriptor l & 15, k = 4s + (l >> 4)),
//   B = 4 k x 16 projections, from an LDS image P'[k][208] (row stride 208
//   = 16 mod 64 banks: the wave's 64 reads hit 64 distinct banks),
//   12 column tiles (188 projections padded to 192 with zeros) per wave tile;
// the signs come out of __ballot per accumulator register.
constexpr int kHashMThreads = 512;
constexpr int kPtStride = 208;

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kHashMThreads) void casc_hash_mfma_kernel(
    const int8_t* __restrict__ desc, const int64_t* __restrict__ img_row0,
    const int32_t* __restrict__ img_n, const int32_t* __restrict__ img_list,
    const float* __restrict__ proj, const float* __restrict__ zm, uint32_t* __restrict__ code,
    uint64_t* __restrict__ bkt) {
    extern __shared__ __attribute__((aligned(16))) float sPt[];   // [128][kPtStride]
    __shared__ float sZ[kCascCode];
    // coalesced reads of proj[p][k], transposed into P'[k][p]; columns 188..207 zero
    for (int i = threadIdx.x; i < kCascProjRows * kCascCode; i += kHashMThreads)
        sPt[(i & (kCascCode - 1)) * kPtStride + (i >> 7)] = proj[i];
    for (int i = threadIdx.x; i < kCascCode * (kPtStride - kCascProjRows); i += kHashMThreads) {
        const int k = i / (kPtStride - kCascProjRows), pj = kCascProjRows + i % (kPtStride - kCascProjRows);
        sPt[k * kPtStride + pj] = 0.f;
    }
    if (threadIdx.x < kCascCode) sZ[threadIdx.x] = zm[threadIdx.x];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int d = lane & 15, j = lane >> 4;
    constexpr int kWaves = kHashMThreads / 64;
    const int I = img_list[blockIdx.y];
    const int n = img_n[I];
    const int64_t row0 = img_row0[I];
    for (int tile = blockIdx.x * kWaves + wave; tile * 16 < n; tile += gridDim.x * kWaves) {
        const int r = min(tile * 16 + d, n - 1);
        // this lane's A column: x[k] for k = 4s + j, s = 0..31
        float x[32];
        const int* src = reinterpret_cast<const int*>(desc + (row0 + r) * 128);
        static_for<32>([&](auto sv) {
            constexpr int sI = decltype(sv)::value;
            const int wv = src[sI];   // bytes 4s .. 4s+3
            const int u = (int)(int8_t)(wv >> (8 * j)) + 128;
            x[sI] = (float)u - sZ[4 * sI + j];
        });
        v4f acc[12];
#pragma unroll
        for (int ct = 0; ct < 12; ++ct) acc[ct] = v4f{0.f, 0.f, 0.f, 0.f};
        static_for<32>([&](auto sv) {
            constexpr int sI = decltype(sv)::value;
            const float* brow = sPt + (4 * sI + j) * kPtStride + d;
            float bv[12];
#pragma unroll
            for (int ct = 0; ct < 12; ++ct) bv[ct] = brow[16 * ct];
#pragma unroll
            for (int ct = 0; ct < 12; ++ct)
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[sI], bv[ct], acc[ct], 0, 0, 0);
            asm volatile("" ::: "memory");   // keep each k-step's 12 LDS reads beside its MFMAs
        });
        // acc[ct][q] = projection 16 ct + (lane & 15) of descriptor 4 (lane >> 4) + q;
        // lane t < 16 collects descriptor t = 4 g + q from the 64-bit ballots
        const int g = (lane >> 2) & 3, q = lane & 3, sh = 16 * g;
        uint32_t cw[4] = {0, 0, 0, 0};
        uint64_t sec = 0;
#pragma unroll
        for (int ct = 0; ct < 12; ++ct) {
            uint32_t mine = 0;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const uint64_t bl = __ballot(acc[ct][qq] > 0.f);
                if (q == qq) mine = (uint32_t)(bl >> sh) & 0xffffu;
            }
            if (ct < 8) cw[ct >> 1] |= mine << (16 * (ct & 1));
            else sec |= (uint64_t)mine << (16 * (ct - 8));
        }
        if (lane < 16 && tile * 16 + lane < n) {
            uint64_t b = 0;
#pragma unroll
            for (int gg = 0; gg < kCascGroups; ++gg) {
                uint32_t id = 0;
#pragma unroll
                for (int k = 0; k < kCascBucketBits; ++k)
                    id = (id << 1) | (uint32_t)((sec >> (gg * kCascBucketBits + k)) & 1);
                b |= (uint64_t)id << (kCascBucketBits * gg);
            }
            const int64_t row = row0 + tile * 16 + lane;
            reinterpret_cast<uint4*>(code)[row] = make_uint4(cw[0], cw[1], cw[2], cw[3]);
            bkt[row] = b;
        }
    }
}

// One wave per (image, group): counting sort of the image's descriptors by
// bucket id; within a bucket the ids stay ascending (the order OpenMVG's
// push_back over j = 0..n-1 leaves them in).
__device__ __forceinline__ int bucket_of(uint64_t b, int g) {
    return (int)(b >> (kCascBucketBits * g)) & (kCascBuckets - 1);
}

__global__ __launch_bounds__(64) void casc_bucket_kernel(const uint64_t* __restrict__ bkt,
                                                         const int64_t* __restrict__ img_row0,
                                                         const int32_t* __restrict__ img_n,
                                                         const int32_t* __restrict__ img_list,
                                                         int64_t rows, int32_t* __restrict__ boff,
                                                         int32_t* __restrict__ blist) {
    const int g = blockIdx.x, I = img_list[blockIdx.y], lane = threadIdx.x;
    __shared__ int hist[kCascBuckets];
    for (int b = lane; b < kCascBuckets; b += 64) hist[b] = 0;
    __syncthreads();
    const int n = img_n[I];
    const int64_t row0 = img_row0[I];
    for (int r = lane; r < n; r += 64) atomicAdd(&hist[bucket_of(bkt[row0 + r], g)], 1);
    __syncthreads();
    int loc[16], s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) { loc[k] = s; s += hist[16 * lane + k]; }
    int incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    const int excl = incl - s;
    int32_t* off = boff + ((int64_t)I * kCascGroups + g) * (kCascBuckets + 1);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        hist[16 * lane + k] = excl + loc[k];
        off[16 * lane + k] = excl + loc[k];
    }
    if (lane == 63) off[kCascBuckets] = incl;
    __syncthreads();
    int32_t* dst = blist + (int64_t)g * rows + row0;
    for (int base = 0; base < n; base += 64) {
        const int r = base + lane;
        const bool valid = r < n;
        const int b = valid ? bucket_of(bkt[row0 + r], g) : 0;
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < kCascBucketBits; ++bit) {
            const bool on = (b >> bit) & 1;
            const uint64_t bb = __ballot(on);
            m &= on ? bb : ~bb;
        }
        const int rank = __popcll(m & ((1ull << lane) - 1));
        int pos = 0;
        if (valid) pos = hist[b] + rank;
        __syncthreads();  // every lane has read its cursor before the leaders move it
        if (valid) {
            dst[pos] = r;
            if (rank == 0) hist[b] += __popcll(m);
        }
        __syncthreads();
    }
}

// Bucket tables of the database image, read from global memory (L2) ...
struct GlobalTabs {
    const int32_t* list;   // blist + row0I; group g at g * rows
    int64_t rows;
    const int32_t* off;    // [6][1025] of image I
    const uint4* code;     // codes of image I
    const uint64_t* bk;    // bucket ids of image I
    __device__ __forceinline__ int at(int g, int e) const { return list[(int64_t)g * rows + e]; }
    __device__ __forceinline__ int bucket(int g, int b) const { return off[g * (kCascBuckets + 1) + b]; }
    __device__ __forceinline__ uint4 cd(int c) const { return code[c]; }
    __device__ __forceinline__ uint64_t bid(int c) const { return bk[c]; }
};
// ... or staged in LDS once per workgroup (u16 ids: images of < 65536 rows)
struct LdsTabs {
    const uint16_t* list;  // [6][n]
    int n;
    const uint16_t* off;   // [6][1025]
    const uint4* code;     // [n]
    const uint64_t* bk;    // [n]
    __device__ __forceinline__ int at(int g, int e) const { return list[g * n + e]; }
    __device__ __forceinline__ int bucket(int g, int b) const { return off[g * (kCascBuckets + 1) + b]; }
    __device__ __forceinline__ uint4 cd(int c) const { return code[c]; }
    __device__ __forceinline__ uint64_t bid(int c) const { return bk[c]; }
};

// One query q (row qrow of image J) against database image I (first row
// row0I): Match_HashedDescriptions + NNdistanceRatio for that query.
//   * candidate c of group g was collected before iff it shares the query's
//     bucket in an earlier group g2 (bucket lists hold every descriptor once
//     per group), so first occurrences are found by comparing bucket ids;
//   * the stable Hamming ranking is a sort on the packed key
//     (h << 24) | (g << 21) | e, e = position in group g's list: arrival
//     order is (g, e) order; the ten smallest keys are kept by a min/max
//     network (2 VALU per slot) and mapped back to ids at the end.
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

template <class T>
__device__ __forceinline__ int casc_collect(const T& tb, const CascMatchArgs& a, int64_t qrow,
                                            uint32_t (&key)[kCascTop]) {
    // returns the number of distinct candidates (0 when <= 2 were collected)
    const uint64_t qb = a.t.bkt[qrow];
    int lo[kCascGroups], hi[kCascGroups], total = 0;
#pragma unroll
    for (int g = 0; g < kCascGroups; ++g) {
        const int b = bucket_of(qb, g);
        lo[g] = tb.bucket(g, b);
        hi[g] = tb.bucket(g, b + 1);
        total += hi[g] - lo[g];
    }
#pragma unroll
    for (int k = 0; k < kCascTop; ++k) key[k] = 0xffffffffu;
    int uniq = 0;
    if (total > 2) {   // candidate_descriptors.size() <= NN: skip
        const uint4 qc = reinterpret_cast<const uint4*>(a.t.code)[qrow];
        // software pipeline per group: the id of entry e+2 and the code /
        // bucket ids of entry e+1 are read while entry e is ranked, so the
        // two dependent LDS round trips per candidate overlap the VALU work
#pragma unroll
        for (int g = 0; g < kCascGroups; ++g) {
            const int e0 = lo[g], e1 = hi[g];
            if (e0 >= e1) continue;
            int c = tb.at(g, e0);
            int cn = e0 + 1 < e1 ? tb.at(g, e0 + 1) : c;
            uint4 cc = tb.cd(c);
            uint64_t cb = tb.bid(c);
            for (int e = e0; e < e1; ++e) {
                const int c1 = cn;
                const uint4 cc1 = tb.cd(c1);
                const uint64_t cb1 = g > 0 ? tb.bid(c1) : 0;
                cn = e + 2 < e1 ? tb.at(g, e + 2) : c1;
                bool dup = false;
#ifndef CASC_DIAG_NODEDUP   // A/B diagnostic builds only
                if (g > 0) {
#else
                if (false) {
#endif
                    const uint64_t x = cb ^ qb;
#pragma unroll
                    for (int g2 = 0; g2 < g; ++g2) dup = dup || bucket_of(x, g2) == 0;
                }
                if (!dup) {
                    ++uniq;
                    const uint32_t h = __popc(qc.x ^ cc.x) + __popc(qc.y ^ cc.y) + __popc(qc.z ^ cc.z) +
                                       __popc(qc.w ^ cc.w);
                    const uint32_t kk = (h << 24) | ((uint32_t)g << 21) | (uint32_t)e;
                    // sorted insertion, one VALU per slot: the new k-th smallest
                    // of {key, kk} is med3(key[k-1], kk, key[k]) (keys ascending),
                    // so updating from the top down reads only old neighbours
#pragma unroll
                    for (int k = kCascTop - 1; k > 0; --k) key[k] = umed3(key[k - 1], kk, key[k]);
                    key[0] = min(key[0], kk);
                }
                c = c1;
                cc = cc1;
                cb = cb1;
            }
        }
    }
    return uniq;
}

template <class T>
__device__ __forceinline__ int key_id(const T& tb, uint32_t key) {
    return tb.at((int)(key >> 21) & 7, (int)(key & 0x1fffff));
}

// partial_sort of (distance, id) pairs + NNdistanceRatio
struct Best2 {
    int d1 = INT_MAX, c1 = INT_MAX, d2 = INT_MAX, c2 = INT_MAX;
    __device__ __forceinline__ void add(int d, int c) {
        if (d < d1 || (d == d1 && c < c1)) {
            d2 = d1; c2 = c1; d1 = d; c1 = c;
        } else if (d < d2 || (d == d2 && c < c2)) {
            d2 = d; c2 = c;
        }
    }
};

// One query q (row qrow of image J) against database image I (first row
// row0I), every lane on its own: Match_HashedDescriptions + NNdistanceRatio.
template <class T>
__device__ __forceinline__ void casc_query(const T& tb, const CascMatchArgs& a, int64_t qrow,
                                           int64_t row0I, int64_t o) {
    uint32_t key[kCascTop];
    const int uniq = casc_collect(tb, a, qrow, key);
    int idx = -1, dd = -1;
    if (uniq >= 2) {
        // rows of the re-ranked candidates: ids and norms first, then the
        // 128-byte rows double-buffered (loads of k+1 in flight during the
        // dot product of k; slots past uniq re-read candidate 0, unused)
        int cid[kCascTop], cn[kCascTop];
#pragma unroll
        for (int k = 0; k < kCascTop; ++k) cid[k] = key_id(tb, key[k < uniq ? k : 0]);
#pragma unroll
        for (int k = 0; k < kCascTop; ++k) cn[k] = a.t.nrm[row0I + cid[k]];
        const int4* qd = reinterpret_cast<const int4*>(a.t.desc + qrow * 128);
        int4 qv[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) qv[w] = qd[w];
        const int nq = a.t.nrm[qrow];
        Best2 b;
        int4 cur[8];
        {
            const int4* cd = reinterpret_cast<const int4*>(a.t.desc + (row0I + cid[0]) * 128);
#pragma unroll
            for (int w = 0; w < 8; ++w) cur[w] = cd[w];
        }
#pragma unroll
        for (int k = 0; k < kCascTop; ++k) {
            int4 nxt[8];
            if (k + 1 < kCascTop) {
                const int4* cd = reinterpret_cast<const int4*>(a.t.desc + (row0I + cid[k + 1]) * 128);
#pragma unroll
                for (int w = 0; w < 8; ++w) nxt[w] = cd[w];
            }
            int dot = 0;
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                dot = __builtin_amdgcn_sdot4(qv[w].x, cur[w].x, dot, false);
                dot = __builtin_amdgcn_sdot4(qv[w].y, cur[w].y, dot, false);
                dot = __builtin_amdgcn_sdot4(qv[w].z, cur[w].z, dot, false);
                dot = __builtin_amdgcn_sdot4(qv[w].w, cur[w].w, dot, false);
            }
            if (k < uniq) b.add(nq + cn[k] - 2 * dot, cid[k]);
            if (k + 1 < kCascTop) {
#pragma unroll
                for (int w = 0; w < 8; ++w) cur[w] = nxt[w];
            }
        }
        if ((float)b.d1 < a.r2 * (float)b.d2) { idx = b.c1; dd = b.d1; }
    }
    a.out_idx[o] = idx;
    a.out_d[o] = dd;
}

__device__ __forceinline__ int xcd_work(int bid, int nwg) {
    // XCD-aware bijective remap of the flat workgroup id (as match_top2_kernel):
    // each XCD gets a contiguous range of work items, so the pairs of one
    // database image share that XCD's L2
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

// Tables of I from global memory: one thread per query, kCascQB per workgroup.
__global__ __launch_bounds__(kCascQB) void casc_match_kernel(CascMatchArgs a) {
    const int work = xcd_work(blockIdx.x, gridDim.x);
    const int pair = work / a.qblocks;
    const int qblk = work - pair * a.qblocks;
    if (pair >= a.n_pairs) return;
    const int I = a.pairs[2 * pair], J = a.pairs[2 * pair + 1];
    const int q = qblk * kCascQB + threadIdx.x;
    if (q >= a.t.img_n[J]) return;
    const int64_t row0I = a.t.img_row0[I];
    GlobalTabs tb{a.t.blist + row0I, a.t.rows,
                  a.t.boff + (int64_t)I * kCascGroups * (kCascBuckets + 1),
                  reinterpret_cast<const uint4*>(a.t.code) + row0I, a.t.bkt + row0I};
    casc_query(tb, a, a.t.img_row0[J] + q, row0I, (int64_t)pair * a.out_stride + q);
}

// Tables of I staged in LDS: one workgroup per pair, every query of J.
__global__ __launch_bounds__(kCascLdsThreads) void casc_match_lds_kernel(CascMatchArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint4 smem[];
    const int pair = xcd_work(blockIdx.x, gridDim.x);
    if (pair >= a.n_pairs) return;
    const int I = a.pairs[2 * pair], J = a.pairs[2 * pair + 1];
    const int nI = a.t.img_n[I], nJ = a.t.img_n[J];
    const int64_t row0I = a.t.img_row0[I];
    uint4* sCode = smem;
    uint64_t* sBk = reinterpret_cast<uint64_t*>(sCode + nI);
    uint16_t* sList = reinterpret_cast<uint16_t*>(sBk + nI);
    uint16_t* sOff = sList + kCascGroups * nI;
    const uint4* gCode = reinterpret_cast<const uint4*>(a.t.code) + row0I;
    for (int i = threadIdx.x; i < nI; i += kCascLdsThreads) {
        sCode[i] = gCode[i];
        sBk[i] = a.t.bkt[row0I + i];
    }
    for (int g = 0; g < kCascGroups; ++g) {
        const int32_t* L = a.t.blist + (int64_t)g * a.t.rows + row0I;
        for (int i = threadIdx.x; i < nI; i += kCascLdsThreads) sList[g * nI + i] = (uint16_t)L[i];
    }
    const int32_t* gOff = a.t.boff + (int64_t)I * kCascGroups * (kCascBuckets + 1);
    for (int i = threadIdx.x; i < kCascGroups * (kCascBuckets + 1); i += kCascLdsThreads)
        sOff[i] = (uint16_t)gOff[i];
    __syncthreads();
    LdsTabs tb{sList, nI, sOff, sCode, sBk};
    const int64_t qrow0 = a.t.img_row0[J];
    for (int q = threadIdx.x; q < nJ; q += kCascLdsThreads)
        casc_query(tb, a, qrow0 + q, row0I, (int64_t)pair * a.out_stride + q);
}

}  // namespace

void casc_colsum(const CascTables& t, int n_img, int64_t* colsum, hipStream_t s) {
    if (n_img == 0) return;
    hipLaunchKernelGGL(casc_colsum_kernel, dim3(n_img), dim3(128), 0, s, t.desc, t.img_row0,
                       t.img_n, colsum);
    SFM_HIP(hipGetLastError());
}

void casc_hash(const CascTables& t, const float* proj, const float* zm, const int32_t* img, int n,
               int max_n, hipStream_t s) {
    if (n == 0 || max_n == 0) return;
    SFM_REQUIRE(n <= 65535, SFM_ERR_UNSUPPORTED, "cascade hashing over %d images", n);
    {
        const size_t mlds = (size_t)kCascCode * kPtStride * sizeof(float);
        set_dyn_lds((const void*)casc_hash_mfma_kernel, mlds);
        // every workgroup stages the 106 KB projection image once: enough
        // workgroups to fill the chip (~1024), not one per 8 tiles
        const int tiles = (max_n + 15) / 16;
        const int per_wg = kHashMThreads / 64;
        const int gx = std::max(1, std::min((tiles + per_wg - 1) / per_wg, std::max(1, 1024 / n)));
        hipLaunchKernelGGL(casc_hash_mfma_kernel, dim3(gx, n), dim3(kHashMThreads), mlds, s, t.desc,
                           t.img_row0, t.img_n, img, proj, zm, t.code, t.bkt);
    }
    SFM_HIP(hipGetLastError());
    hipLaunchKernelGGL(casc_bucket_kernel, dim3(kCascGroups, n), dim3(64), 0, s, t.bkt, t.img_row0,
                       t.img_n, img, t.rows, t.boff, t.blist);
    SFM_HIP(hipGetLastError());
}

size_t casc_lds_bytes(int max_n) {
    return (size_t)max_n * (16 + 8 + 2 * kCascGroups) + (size_t)kCascGroups * (kCascBuckets + 1) * 2;
}

void casc_match(const CascMatchArgs& a, int max_n, hipStream_t s) {
    if (a.n_pairs == 0) return;
    const size_t lds = casc_lds_bytes(max_n);
    if (max_n <= kCascLdsMaxN) {
        set_dyn_lds((const void*)casc_match_lds_kernel, casc_lds_bytes(kCascLdsMaxN));
        hipLaunchKernelGGL(casc_match_lds_kernel, dim3((unsigned)a.n_pairs), dim3(kCascLdsThreads),
                           lds, s, a);
    } else {
        const int64_t nwg = (int64_t)a.n_pairs * a.qblocks;
        hipLaunchKernelGGL(casc_match_kernel, dim3((unsigned)nwg), dim3(kCascQB), 0, s, a);
    }
    SFM_HIP(hipGetLastError());
}

}  // namespace sfm
