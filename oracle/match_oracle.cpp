// CPU restatement of the reference's descriptor matchers — TEST
// INFRASTRUCTURE ONLY (see oracle.h; parity unpinned).
//
// RATIO  (src/sparseBuilder/sparseBuilder.cpp:919-921, fDistRatio :812):
//   OpenMVG Matcher_Regions(BRUTE_FORCE_L2) builds the matcher on regions I
//   and queries it with regions J; for every query j the two nearest database
//   entries (squared L2, exact for uchar) d1 <= d2 are found and the match
//   IndMatch(i = nn index, j) is kept iff d1 < fl32(ratio^2) * d2 (OpenMVG
//   NNdistanceRatio with Square(f_dist_ratio)).  Ties: lowest database index
//   wins (documented choice; OpenMVG's partial_sort leaves it unspecified).
//   Pairs with fewer than 2 database entries give no matches.  Output order:
//   sorted by (i, j) (IndMatch::getDeduplicated).
// MUTUAL (src/frame/LocalFrame.h:31-47, GlobalFrame.h:22-43 with
//   cv::BFMatcher(NORM_L2, crossCheck=true), SequentialActuator.h:77):
//   keep (q, t) iff t = argmin_t d(q, .) and q = argmin_q d(., t); first
//   minimum (lowest index) wins.  Integer d ordering equals OpenCV's
//   fl32(sqrt(d)) ordering for d < 2^22, which covers 512-normalised SIFT.
#include <algorithm>
#include <cmath>
#include <climits>
#include <cstdint>
#include <cstring>
#include <vector>

#include "oracle.h"

namespace {

inline int32_t l2sq(const uint8_t* a, const uint8_t* b) {
    int32_t s = 0;
    for (int k = 0; k < 128; ++k) {
        const int32_t d = (int32_t)a[k] - (int32_t)b[k];
        s += d * d;
    }
    return s;
}

// For every row of q: best and second-best (value) over rows of db.
void top2(const uint8_t* db, int32_t n_db, const uint8_t* q, int32_t n_q,
          int32_t* best_idx, int32_t* best_d, int32_t* second_d, int n_threads = 1) {
#pragma omp parallel for schedule(static, 64) num_threads(n_threads > 0 ? n_threads : 1) if (n_threads > 1)
    for (int32_t t = 0; t < n_q; ++t) {
        int32_t b1 = INT32_MAX, b2 = INT32_MAX, i1 = -1;
        const uint8_t* qt = q + (int64_t)t * 128;
        for (int32_t s = 0; s < n_db; ++s) {
            const int32_t d = l2sq(db + (int64_t)s * 128, qt);
            if (d < b1) { b2 = b1; b1 = d; i1 = s; }
            else if (d < b2) { b2 = d; }
        }
        best_idx[t] = i1; best_d[t] = b1;
        if (second_d) second_d[t] = b2;
    }
}

}  // namespace

extern "C" int orc_match_dense(const uint8_t* a, int32_t n_a, const uint8_t* b, int32_t n_b,
                               int32_t mode, float ratio, int32_t* match_idx,
                               int32_t* match_d2) {
    return orc_match_dense_mt(a, n_a, b, n_b, mode, ratio, 1, match_idx, match_d2);
}

extern "C" int orc_match_dense_mt(const uint8_t* a, int32_t n_a, const uint8_t* b, int32_t n_b,
                                  int32_t mode, float ratio, int32_t n_threads, int32_t* match_idx,
                                  int32_t* match_d2) {
    if (n_a < 0 || n_b < 0) return SFM_ERR_INVALID_ARG;
    if (mode == SFM_MATCH_RATIO) {
        std::vector<int32_t> bi(n_b), bd(n_b), sd(n_b);
        top2(a, n_a, b, n_b, bi.data(), bd.data(), sd.data(), n_threads);
        const float r2 = ratio * ratio;  // Square(f_dist_ratio) in float
        for (int32_t t = 0; t < n_b; ++t) {
            bool keep = n_a >= 2 && (float)bd[t] < r2 * (float)sd[t];
            match_idx[t] = keep ? bi[t] : -1;
            match_d2[t] = keep ? bd[t] : -1;
        }
        return SFM_OK;
    }
    if (mode == SFM_MATCH_MUTUAL) {
        std::vector<int32_t> nq(n_a), dq(n_a), nt(n_b), dt(n_b);
        top2(b, n_b, a, n_a, nq.data(), dq.data(), nullptr, n_threads);  // per query row of a
        top2(a, n_a, b, n_b, nt.data(), dt.data(), nullptr, n_threads);  // per train row of b
        for (int32_t q = 0; q < n_a; ++q) {
            const int32_t t = nq[q];
            const bool keep = t >= 0 && nt[t] == q;
            match_idx[q] = keep ? t : -1;
            match_d2[q] = keep ? dq[q] : -1;
        }
        return SFM_OK;
    }
    if (mode == SFM_MATCH_CASCADE) {   // a 2-image collection, pair (0, 1)
        std::vector<uint8_t> d((size_t)(n_a + n_b) * 128);
        if (n_a) std::memcpy(d.data(), a, (size_t)n_a * 128);
        if (n_b) std::memcpy(d.data() + (size_t)n_a * 128, b, (size_t)n_b * 128);
        const int64_t off[3] = {0, n_a, (int64_t)n_a + n_b};
        const int32_t pair[2] = {0, 1};
        return orc_cascade_pairs(d.data(), off, 2, pair, 1, ratio, 1, std::max(1, n_b), match_idx,
                                 match_d2);
    }
    return SFM_ERR_INVALID_ARG;
}

// Float descriptors (cv::Mat CV_32F, LocalFrame.h:38): d = sum_k (a_k - b_k)^2
// as an fmaf chain in k order, top-2 / first minimum as for u8.  For integer
// values in [0, 255] every order gives the same exact integer (< 2^24), which
// is OpenCV's result; for other values this order is the restatement's own
// (OpenCV's SIMD summation order is not pinned here).
namespace {
inline float l2sq_f32(const float* a, const float* b) {
    float s = 0.f;
    for (int k = 0; k < 128; ++k) {
        const float t = a[k] - b[k];
        s = std::fmaf(t, t, s);
    }
    return s;
}
void top2_f32(const float* db, int32_t n_db, const float* q, int32_t n_q, int32_t* best_idx, float* best_d,
              float* second_d, int n_threads) {
#pragma omp parallel for schedule(static, 64) num_threads(n_threads > 0 ? n_threads : 1) if (n_threads > 1)
    for (int32_t t = 0; t < n_q; ++t) {
        float b1 = INFINITY, b2 = INFINITY;
        int32_t i1 = -1;
        const float* qt = q + (int64_t)t * 128;
        for (int32_t s = 0; s < n_db; ++s) {
            const float d = l2sq_f32(qt, db + (int64_t)s * 128);
            if (d < b1) { b2 = b1; b1 = d; i1 = s; }
            else if (d < b2) { b2 = d; }
        }
        best_idx[t] = i1; best_d[t] = b1;
        if (second_d) second_d[t] = b2;
    }
}
}  // namespace

extern "C" int orc_match_dense_f32(const float* a, int32_t n_a, const float* b, int32_t n_b, int32_t mode,
                                   float ratio, int32_t n_threads, int32_t* match_idx, float* match_d2) {
    if (n_a < 0 || n_b < 0) return SFM_ERR_INVALID_ARG;
    if (mode == SFM_MATCH_RATIO) {
        std::vector<int32_t> bi(n_b);
        std::vector<float> bd(n_b), sd(n_b);
        top2_f32(a, n_a, b, n_b, bi.data(), bd.data(), sd.data(), n_threads);
        const float r2 = ratio * ratio;
        for (int32_t t = 0; t < n_b; ++t) {
            const bool keep = n_a >= 2 && bd[t] < r2 * sd[t];
            match_idx[t] = keep ? bi[t] : -1;
            match_d2[t] = keep ? bd[t] : -1.f;
        }
        return SFM_OK;
    }
    if (mode == SFM_MATCH_MUTUAL) {
        std::vector<int32_t> nq(n_a), nt(n_b);
        std::vector<float> dq(n_a), dt(n_b);
        top2_f32(b, n_b, a, n_a, nq.data(), dq.data(), nullptr, n_threads);
        top2_f32(a, n_a, b, n_b, nt.data(), dt.data(), nullptr, n_threads);
        for (int32_t q = 0; q < n_a; ++q) {
            const int32_t t = nq[q];
            const bool keep = t >= 0 && nt[t] == q;
            match_idx[q] = keep ? t : -1;
            match_d2[q] = keep ? dq[q] : -1.f;
        }
        return SFM_OK;
    }
    return SFM_ERR_UNSUPPORTED;
}

extern "C" int orc_match_pairs(const uint8_t* desc, const int64_t* offsets, int32_t n_img,
                               const int32_t* pairs, int64_t n_pairs, int32_t mode,
                               float ratio, int32_t n_threads, int64_t* counts, uint32_t* i,
                               uint32_t* j, int32_t* d2) {
    if (n_pairs < 0 || !counts) return SFM_ERR_INVALID_ARG;
    std::vector<std::vector<std::pair<uint64_t, int32_t>>> res(n_pairs);
    int err = SFM_OK;
    if (mode == SFM_MATCH_CASCADE) {   // hashing needs the whole pair list at once
        int64_t stride = 1;
        for (int32_t k = 0; k < n_img; ++k) stride = std::max(stride, offsets[k + 1] - offsets[k]);
        std::vector<int32_t> idx((size_t)(n_pairs * stride)), dd((size_t)(n_pairs * stride));
        const int e = orc_cascade_pairs(desc, offsets, n_img, pairs, n_pairs, ratio, n_threads,
                                        stride, idx.data(), dd.data());
        if (e) return e;
        for (int64_t p = 0; p < n_pairs; ++p) {
            const int32_t J = pairs[2 * p + 1];
            for (int64_t t = 0; t < offsets[J + 1] - offsets[J]; ++t)
                if (idx[p * stride + t] >= 0)
                    res[p].emplace_back(((uint64_t)(uint32_t)idx[p * stride + t] << 32) | (uint32_t)t,
                                        dd[p * stride + t]);
            std::sort(res[p].begin(), res[p].end());
        }
    } else {
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads > 0 ? n_threads : 1)
        for (int64_t p = 0; p < n_pairs; ++p) {
            const int32_t I = pairs[2 * p], J = pairs[2 * p + 1];
            if (I < 0 || J < 0 || I >= n_img || J >= n_img) { err = SFM_ERR_INVALID_ARG; continue; }
            const int32_t nI = (int32_t)(offsets[I + 1] - offsets[I]);
            const int32_t nJ = (int32_t)(offsets[J + 1] - offsets[J]);
            const uint8_t* dI = desc + offsets[I] * 128;
            const uint8_t* dJ = desc + offsets[J] * 128;
            const int32_t n_out = mode == SFM_MATCH_RATIO ? nJ : nI;
            std::vector<int32_t> idx(n_out), dd(n_out);
            orc_match_dense(dI, nI, dJ, nJ, mode, ratio, idx.data(), dd.data());
            auto& v = res[p];
            for (int32_t t = 0; t < n_out; ++t) {
                if (idx[t] < 0) continue;
                const uint32_t ii = mode == SFM_MATCH_RATIO ? (uint32_t)idx[t] : (uint32_t)t;
                const uint32_t jj = mode == SFM_MATCH_RATIO ? (uint32_t)t : (uint32_t)idx[t];
                v.emplace_back(((uint64_t)ii << 32) | jj, dd[t]);
            }
            std::sort(v.begin(), v.end());
        }
    }
    if (err) return err;
    int64_t off = 0;
    for (int64_t p = 0; p < n_pairs; ++p) {
        counts[p] = (int64_t)res[p].size();
        if (i) {
            for (const auto& m : res[p]) {
                i[off] = (uint32_t)(m.first >> 32);
                j[off] = (uint32_t)(m.first & 0xffffffffu);
                d2[off] = m.second;
                ++off;
            }
        }
    }
    return SFM_OK;
}

// OpenMVG IndMatchDecorator<float>::getDeduplicated (matching/
// indMatchDecoratorXY.hpp, un-vendored; parity unpinned): the (i, j)-sorted
// matches, decorated with (xI, yI, xJ, yJ), are copied into a std::set keyed
// by the decorator's operator<; the set's iteration order is the result.
// That operator< is the upstream one verbatim in meaning: equal coordinates
// compare false; otherwise a differing x1 only selects a y1 comparison, and
// an equal x1 requires both x2 and y2 to be smaller.
namespace {
struct OrcDecorated {
    float x1, y1, x2, y2;
    uint32_t i, j;
    friend bool operator==(const OrcDecorated& m1, const OrcDecorated& m2) {
        return m1.x1 == m2.x1 && m1.y1 == m2.y1 && m1.x2 == m2.x2 && m1.y2 == m2.y2;
    }
    friend bool operator<(const OrcDecorated& m1, const OrcDecorated& m2) {
        if (m1 == m2) return false;
        if (m1.x1 < m2.x1)
            return m1.y1 < m2.y1;
        else if (m1.x1 > m2.x1)
            return m1.y1 < m2.y1;
        return m1.x2 < m2.x2 && m1.y2 < m2.y2;
    }
};
}  // namespace

#include <set>
extern "C" int orc_dedup_decorator(const uint32_t* i, const uint32_t* j, int64_t n, const float* feat_i,
                                   const float* feat_j, uint32_t* out_i, uint32_t* out_j, int64_t* n_out) {
    if ((n > 0 && (!i || !j || !feat_i || !feat_j || !out_i || !out_j)) || !n_out) return SFM_ERR_INVALID_ARG;
    std::vector<OrcDecorated> v;
    for (int64_t k = 0; k < n; ++k)
        v.push_back(OrcDecorated{feat_i[4 * (size_t)i[k]], feat_i[4 * (size_t)i[k] + 1], feat_j[4 * (size_t)j[k]],
                                 feat_j[4 * (size_t)j[k] + 1], i[k], j[k]});
    std::set<OrcDecorated> s(v.begin(), v.end());
    int64_t w = 0;
    for (const auto& d : s) { out_i[w] = d.i; out_j[w] = d.j; ++w; }
    *n_out = w;
    return SFM_OK;
}
