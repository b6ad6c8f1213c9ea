// Cascade-hashing matcher (SFM_MATCH_CASCADE): launch wrappers for
// cascade.hip, driven by the match plan in match.hip.
//
// Reference: src/sparseBuilder/sparseBuilder.cpp:811-814,911-914 — "AUTO" on
// uchar SIFT regions selects OpenMVG Cascade_Hashing_Matcher_Regions(0.8),
// the live default of the reference pipeline.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace sfm {

constexpr int kCascCode = 128;      // primary hash bits (= descriptor length)
constexpr int kCascGroups = 6;      // bucket groups
constexpr int kCascBucketBits = 10; // bits per bucket id
constexpr int kCascBuckets = 1 << kCascBucketBits;
constexpr int kCascTop = 10;        // candidates re-ranked by exact L2 per query
constexpr int kCascProjRows = kCascCode + kCascGroups * kCascBucketBits;  // 188

// CascadeHasher::Init: std::mt19937(default_seed), std::normal_distribution<>
// (0,1) draws, primary 128x128 row by row, then the 6 secondary 10x128
// matrices; stored as float [188][128].
void casc_projections(std::vector<float>& proj);

// Zero-mean descriptor of Cascade_Hashing_Matcher_Regions: the mean over the
// used images of each image's column mean.  colsum[n_img][128] are exact
// per-image column sums of the uint8 descriptors.
void casc_zero_mean(const int64_t* colsum, const int32_t* img_n, const std::vector<int32_t>& used,
                    float* zm);

struct CascTables {
    const int8_t* desc;       // padded rows x 128, a - 128 (match plan layout)
    const int32_t* nrm;       // |a - 128|^2 per row
    const int64_t* img_row0;  // first padded row per image
    const int32_t* img_n;     // rows per image
    int64_t rows;             // padded rows in total
    uint32_t* code;           // [rows][4]   128-bit hash code
    uint64_t* bkt;            // [rows]      6 bucket ids, group g in bits [10g, 10g+10)
    int32_t* boff;            // [n_img][6][1025] bucket start per image and group
    int32_t* blist;           // [6][rows]   descriptor ids per bucket, ascending
};

void casc_colsum(const CascTables& t, int n_img, int64_t* colsum, hipStream_t s);
// Hash codes and bucket ids of every descriptor of the images in img[n],
// then their bucket lists.
void casc_hash(const CascTables& t, const float* proj, const float* zm, const int32_t* img,
               int n, int max_n, hipStream_t s);

struct CascMatchArgs {
    CascTables t;
    const int32_t* pairs;     // (I, J): database I, queries J
    int32_t n_pairs;
    int32_t qblocks;
    float r2;                 // fl32(ratio^2)
    int64_t out_stride;
    int32_t* out_idx;         // per query of J: matched row of I or -1
    int32_t* out_d;           // its squared L2 distance or -1
};
constexpr int kCascQB = 256;          // queries per workgroup (tables in global memory)
constexpr int kCascLdsThreads = 1024; // one workgroup per pair (tables in LDS)
constexpr int kCascLdsMaxN = 4200;    // largest image whose tables fit 160 KB of LDS
// max_n: most rows of any image; picks the LDS-staged kernel when it fits
void casc_match(const CascMatchArgs& a, int max_n, hipStream_t s);

}  // namespace sfm
