// Host planning for the BA kernels: active parameter blocks (the reduced
// program Ceres builds: constant and unobserved blocks removed), reduced
// camera system (RCS) ordering, landmark partition across ranks, Schur work
// chunks (camera windows that fit one 80-row MFMA tile), and the static
// gather plan that sums chunk tiles and per-image blocks into the banded RCS.
//
// Reference: BundleAdjuster.h:100-123 builds the problem (pose blocks 6,
// intrinsic blocks 4, point blocks 3, one residual block per observation,
// gauge :105); ceres SPARSE_SCHUR eliminates the point blocks.
#include "ba_plan.h"

#include <algorithm>
#include <atomic>
#include <climits>
#include <condition_variable>
#include <exception>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <thread>

#include "common.h"
#include "../include/sfm/pool.hpp"

namespace sfm {

namespace {

// Split [0, n) into contiguous ranges over up to 16 host threads (results are
// independent of the split: every range writes its own outputs).
template <class F>
void parallel_ranges(int64_t n, F&& fn) {
    const int64_t nt = n < 4096 ? 1 : std::min<int64_t>(PlanPool::width(), n / 2048);
    if (nt <= 1) {
        fn(0, n, 0);
        return;
    }
    PlanPool::get().run((int)nt, [&](int t) { fn(n * t / nt, n * (t + 1) / nt, t); });
}

// fn(g) for g in [0, nseg) on the host threads (each g writes its own outputs)
template <class F>
void parallel_segments(int nseg, F&& fn) {
    PlanPool::get().run(nseg, [&](int g) { fn(g); });
}

// block half-bandwidth of the points' camera spans under the order cam_blk;
// *lb_out (optional): a bound no camera order can beat, the largest number of
// distinct active cameras one point sees, minus one
// (spans, optional: every point's [first, last + 1) active block, (ncam, 0)
// without one -- partition_points' sort keys, computed in the same pass)
int32_t half_bandwidth(const sfm_ba_problem& P, const std::vector<int32_t>& cam_blk, int32_t* lb_out = nullptr,
                       PointSpans* spans = nullptr, int32_t ncam = 0) {
    int32_t Dt[16] = {0}, Lt[16] = {0};
    if (spans) {
        spans->lo.resize(P.n_pt);
        spans->hi.resize(P.n_pt);
    }
    parallel_ranges(P.n_pt, [&](int64_t p0, int64_t p1, int t) {
        int32_t D = 0, L = 0;
        std::vector<int32_t> cs;
        for (int64_t p = p0; p < p1; ++p) {
            int lo = INT_MAX, hi = -1, n = 0;
            for (int64_t o = P.pt_offsets[p]; o < P.pt_offsets[p + 1]; ++o) {
                const int b = cam_blk[P.obs_img[o]];
                if (b >= 0) { lo = std::min(lo, b); hi = std::max(hi, b); ++n; }
            }
            if (hi >= 0) D = std::max(D, hi - lo);
            if (spans) {
                spans->lo[p] = hi >= 0 ? lo : ncam;
                spans->hi[p] = hi + 1;
            }
            if (lb_out && n - 1 > L) {   // only a track longer than the bound so far is counted exactly
                cs.clear();
                for (int64_t o = P.pt_offsets[p]; o < P.pt_offsets[p + 1]; ++o)
                    if (cam_blk[P.obs_img[o]] >= 0) cs.push_back(cam_blk[P.obs_img[o]]);
                std::sort(cs.begin(), cs.end());
                L = std::max(L, (int32_t)(std::unique(cs.begin(), cs.end()) - cs.begin()) - 1);
            }
        }
        Dt[t] = D;
        Lt[t] = L;
    });
    int32_t D = 0, L = 0;
    for (int t = 0; t < 16; ++t) { D = std::max(D, Dt[t]); L = std::max(L, Lt[t]); }
    if (lb_out) *lb_out = L;
    return D;
}

// flags[i] = 1 for every value i = idx[o] (o < n): a per-thread pass each
void mark_used(const int32_t* idx, int64_t n, int32_t m, std::vector<char>& flags) {
    std::vector<std::vector<char>> part(16);
    parallel_ranges(n, [&](int64_t o0, int64_t o1, int t) {
        part[t].assign(m, 0);
        for (int64_t o = o0; o < o1; ++o) part[t][idx[o]] = 1;
    });
    flags.assign(m, 0);
    for (const auto& f : part)
        for (int32_t i = 0; i < (int32_t)f.size(); ++i) flags[i] |= f[i];
}

// Reverse Cuthill-McKee over the camera co-visibility graph (cameras that
// share a point are adjacent): a closed orbit, whose first and last images
// see the same points, gets a band of ~2k blocks instead of the whole RCS.
// Long tracks contribute a chain of nearest neighbours only.  Returns the new
// block of every natural block.
std::vector<int32_t> rcm_order(const sfm_ba_problem& P, const std::vector<int32_t>& cam_blk, int32_t ncam) {
    // adjacency rows in ascending neighbour order: a bit matrix while it is
    // small (ncam <= 8192: <= 8 MB), else a sorted, de-duplicated edge list
    std::vector<int64_t> ptr(ncam + 1, 0);
    std::vector<int32_t> adj;
    auto each_pair = [&](auto&& emit) {
        std::vector<int32_t> cs;
        for (int64_t p = 0; p < P.n_pt; ++p) {
            cs.clear();
            for (int64_t o = P.pt_offsets[p]; o < P.pt_offsets[p + 1]; ++o)
                if (cam_blk[P.obs_img[o]] >= 0) cs.push_back(cam_blk[P.obs_img[o]]);
            std::sort(cs.begin(), cs.end());
            cs.erase(std::unique(cs.begin(), cs.end()), cs.end());
            const size_t n = cs.size(), reach = n <= 24 ? n : 4;
            for (size_t a = 0; a < n; ++a)
                for (size_t b = a + 1; b < std::min(n, a + 1 + reach); ++b) emit(cs[a], cs[b]);
        }
    };
    if (ncam <= 8192) {
        const int64_t words = (ncam + 63) / 64;
        std::vector<uint64_t> bits((size_t)(ncam * words), 0);
        each_pair([&](int32_t a, int32_t b) {
            bits[(size_t)(a * words + (b >> 6))] |= 1ull << (b & 63);
            bits[(size_t)(b * words + (a >> 6))] |= 1ull << (a & 63);
        });
        for (int32_t c = 0; c < ncam; ++c) {
            for (int64_t w = 0; w < words; ++w)
                for (uint64_t m = bits[(size_t)(c * words + w)]; m; m &= m - 1)
                    adj.push_back((int32_t)(64 * w + __builtin_ctzll(m)));
            ptr[c + 1] = (int64_t)adj.size();
        }
    } else {
        std::vector<uint64_t> edges;
        each_pair([&](int32_t a, int32_t b) {
            edges.push_back(((uint64_t)a << 32) | (uint32_t)b);
            edges.push_back(((uint64_t)b << 32) | (uint32_t)a);
        });
        std::sort(edges.begin(), edges.end());
        edges.erase(std::unique(edges.begin(), edges.end()), edges.end());
        for (uint64_t e : edges) ptr[(e >> 32) + 1]++;
        for (int32_t c = 0; c < ncam; ++c) ptr[c + 1] += ptr[c];
        adj.resize(edges.size());
        for (size_t k = 0; k < edges.size(); ++k) adj[k] = (int32_t)(edges[k] & 0xffffffffu);
    }
    auto deg = [&](int32_t c) { return ptr[c + 1] - ptr[c]; };
    std::vector<int32_t> seq;
    std::vector<char> seen(ncam, 0);
    auto bfs = [&](int32_t s, std::vector<int32_t>& out, std::vector<char>& mark) {
        out.clear();
        out.push_back(s);
        mark[s] = 1;
        std::vector<int32_t> nb;
        for (size_t h = 0; h < out.size(); ++h) {
            const int32_t c = out[h];
            nb.assign(adj.begin() + ptr[c], adj.begin() + ptr[c + 1]);
            std::stable_sort(nb.begin(), nb.end(), [&](int32_t a, int32_t b) { return deg(a) < deg(b); });
            for (int32_t n : nb)
                if (!mark[n]) { mark[n] = 1; out.push_back(n); }
        }
    };
    std::vector<int32_t> byd(ncam);
    std::iota(byd.begin(), byd.end(), 0);
    std::stable_sort(byd.begin(), byd.end(), [&](int32_t a, int32_t b) { return deg(a) < deg(b); });
    std::vector<int32_t> comp;
    for (int32_t s0 : byd) {
        if (seen[s0]) continue;
        // pseudo-peripheral start: the last-reached node of a BFS from s0
        std::vector<char> tmp(seen);
        bfs(s0, comp, tmp);
        int32_t s = comp.back();
        bfs(s, comp, seen);
        seq.insert(seq.end(), comp.begin(), comp.end());
    }
    std::reverse(seq.begin(), seq.end());
    std::vector<int32_t> newpos(ncam);
    for (int32_t k = 0; k < ncam; ++k) newpos[seq[k]] = k;
    return newpos;
}

}  // namespace

std::vector<int32_t> camera_blocks(const sfm_ba_problem& P, int32_t* ncam_out, int32_t* D_out, PointSpans* spans,
                                   std::vector<char>* used_out, int32_t* lb_out, bool* rcm_out) {
    PhaseTimer tm("camera_blocks");
    if (rcm_out) *rcm_out = false;
    std::vector<int32_t> cam_blk(P.n_img, -1);
    std::vector<char> used;
    mark_used(P.obs_img, P.n_obs, P.n_img, used);
    int32_t ncam = 0;
    for (int i = 0; i < P.n_img; ++i)
        if (used[i] && i != P.const_img) cam_blk[i] = ncam++;
    tm.mark("used");
    int32_t lb = 0;
    int32_t D = half_bandwidth(P, cam_blk, &lb, spans, ncam);
    // reorder only when the image order does not give a band the BCR solver
    // takes, no order can (a point seeing more than kBandMaxD + 1 cameras
    // keeps the RCS dense under any order), and the co-visibility graph is
    // small enough to build quickly
    tm.mark("bandwidth");
    if (D > kBandMaxD && lb <= kBandMaxD && ncam > 2 && P.n_obs <= (int64_t)8 << 20) {
        const std::vector<int32_t> pos = rcm_order(P, cam_blk, ncam);
        tm.mark("rcm");
        std::vector<int32_t> alt(cam_blk);
        for (auto& b : alt)
            if (b >= 0) b = pos[b];
        PointSpans alt_spans;
        const int32_t D2 = half_bandwidth(P, alt, nullptr, spans ? &alt_spans : nullptr, ncam);
        if (D2 < D) {
            cam_blk.swap(alt);
            D = D2;
            if (spans) *spans = std::move(alt_spans);
            if (rcm_out) *rcm_out = true;
        }
        tm.mark("bandwidth2");
    }
    if (lb_out) *lb_out = lb;
    if (ncam_out) *ncam_out = ncam;
    if (D_out) *D_out = D;
    if (used_out) used_out->swap(used);
    return cam_blk;
}

namespace {

// Everything of the active parameter blocks that follows from cam_blk (ncam,
// D set) and the observed-image flags
void active_from_blocks(const sfm_ba_problem& P, BAHostPlan& pl, const std::vector<char>& im) {
    pl.blk_img.assign(pl.ncam, -1);
    for (int i = 0; i < P.n_img; ++i)
        if (pl.cam_blk[i] >= 0) pl.blk_img[pl.cam_blk[i]] = i;
    pl.intr_blk.assign(P.n_intr, -1);
    pl.blk_intr.clear();
    pl.nintr = 0;
    // intrinsics blocks of observed images
    std::vector<char> iu(P.n_intr, 0);
    for (int i = 0; i < P.n_img; ++i)
        if (im[i]) iu[P.img_intr[i]] = 1;
    for (int q = 0; q < P.n_intr; ++q)
        if (iu[q]) { pl.intr_blk[q] = pl.nintr++; pl.blk_intr.push_back(q); }
    pl.iw = sfm_ba_intr_width(P.camera_model);
    pl.nb = 6LL * pl.ncam;
    pl.na = (int64_t)pl.iw * pl.nintr;
    pl.nF = pl.nb + pl.na;
    pl.nFB = pl.ncam + pl.nintr;
    pl.img_colc.assign(P.n_img, -1);
    pl.img_coli.assign(P.n_img, -1);
    pl.img_intr.assign(P.img_intr, P.img_intr + P.n_img);
    for (int i = 0; i < P.n_img; ++i) {
        if (pl.cam_blk[i] >= 0) pl.img_colc[i] = 6 * pl.cam_blk[i];
        const int q = pl.intr_blk[P.img_intr[i]];
        if (q >= 0) pl.img_coli[i] = (int32_t)(pl.nb + (int64_t)pl.iw * q);
    }
}

}  // namespace

void partition_points(const sfm_ba_problem& P, const std::vector<int32_t>& cam_blk, int world,
                      std::vector<int64_t>& order, std::vector<int64_t>& bounds, const PointSpans* spans) {
    // stable order by (first, last) active camera block: two stable counting
    // passes (last, then first) over ncam + 1 buckets (no active camera sorts
    // last), the order std::stable_sort on the pair gives
    int32_t ncam = 0;
    for (int32_t b : cam_blk) ncam = std::max(ncam, b + 1);
    PointSpans own;
    if (!spans) {   // (camera_blocks' pass gives them to build_plan)
        own.lo.resize(P.n_pt);
        own.hi.resize(P.n_pt);
        parallel_ranges(P.n_pt, [&](int64_t p0, int64_t p1, int) {
            for (int64_t p = p0; p < p1; ++p) {
                int l = ncam, h = 0;
                for (int64_t o = P.pt_offsets[p]; o < P.pt_offsets[p + 1]; ++o) {
                    const int b = cam_blk[P.obs_img[o]];
                    if (b >= 0) { l = std::min(l, b); h = std::max(h, b + 1); }
                }
                own.lo[p] = l;
                own.hi[p] = h;
            }
        });
        spans = &own;
    }
    const std::vector<int32_t>& lo = spans->lo;
    const std::vector<int32_t>& hi = spans->hi;
    // each pass a stable counting sort over host ranges: per-range bucket
    // counts, offsets in (bucket, range) order, every range scattering its
    // own items in order -- the serial pass's output
    constexpr int kMaxR = 16;
    const int64_t nr = P.n_pt < 16384 ? 1 : std::min<int64_t>(kMaxR, std::min<int64_t>(PlanPool::width(), P.n_pt / 8192));
    std::vector<int64_t> tmp(P.n_pt), cnt((size_t)nr * (ncam + 2));
    auto pass = [&](const std::vector<int32_t>& key, const int64_t* in, int64_t* out) {
        auto range = [&](int r, int64_t& k0, int64_t& k1) { k0 = P.n_pt * r / nr; k1 = P.n_pt * (r + 1) / nr; };
        std::fill(cnt.begin(), cnt.end(), 0);
        auto count = [&](int r) {
            int64_t k0, k1;
            range(r, k0, k1);
            int64_t* c = &cnt[(size_t)r * (ncam + 2)];
            for (int64_t k = k0; k < k1; ++k) c[key[in ? in[k] : k] + 1]++;
        };
        auto scatter = [&](int r) {
            int64_t k0, k1;
            range(r, k0, k1);
            int64_t* c = &cnt[(size_t)r * (ncam + 2)];
            for (int64_t k = k0; k < k1; ++k) {
                const int64_t p = in ? in[k] : k;
                out[c[key[p]]++] = p;
            }
        };
        if (nr > 1) PlanPool::get().run((int)nr, count);
        else count(0);
        // c[r][b] (after the scan) = first slot of bucket b's items from range r
        int64_t acc = 0;
        for (int32_t b = 0; b <= ncam; ++b)
            for (int r = 0; r < nr; ++r) {
                int64_t& c = cnt[(size_t)r * (ncam + 2) + b + 1];
                const int64_t n = c;
                cnt[(size_t)r * (ncam + 2) + b] = acc;   // slot b holds the start (b + 1 held the count)
                acc += n;
            }
        if (nr > 1) PlanPool::get().run((int)nr, scatter);
        else scatter(0);
    };
    order.resize(P.n_pt);
    pass(hi, nullptr, tmp.data());
    pass(lo, tmp.data(), order.data());
    bounds.assign(world + 1, P.n_pt);
    bounds[0] = 0;
    int64_t acc = 0, r = 1;
    for (int64_t k = 0; k < P.n_pt && r < world; ++k) {
        const int64_t p = order[k];
        acc += P.pt_offsets[p + 1] - P.pt_offsets[p];
        while (r < world && acc * world >= r * P.n_obs) bounds[r++] = k + 1;
    }
}

namespace {

// A point goes through the Schur chunk kernel when its F rows fit a chunk
// tile and its observations one wave batch; everything else is a general
// point (Ceres takes any track length, any number of camera
// intrinsics and repeated (point, image) observations).
bool chunkable(const sfm_ba_problem& P, const BAHostPlan& pl, int64_t p) {
    const int64_t o0 = P.pt_offsets[p], o1 = P.pt_offsets[p + 1];
    if (o1 - o0 > kSubObs) return false;
    int nc = 0, ni = 0;
    int32_t intrs[kIntrSlots];
    for (int64_t o = o0; o < o1; ++o) {
        const int img = P.obs_img[o];
        for (int64_t o2 = o0; o2 < o; ++o2)
            if (P.obs_img[o2] == img) return false;      // the same image twice
        if (pl.cam_blk[img] >= 0) ++nc;
        const int q = P.img_intr[img];
        bool have = false;
        for (int t = 0; t < ni; ++t) have |= intrs[t] == q;
        if (!have) {
            if (ni == kIntrSlots) return false;
            intrs[ni++] = q;
        }
    }
    return o1 - o0 <= kCamSlots && 6 * nc + pl.iw * ni <= kTileRowsUsed;
}

}  // namespace

namespace {

void validate_problem(const sfm_ba_problem& P) {
    SFM_REQUIRE(P.n_img >= 1 && P.n_intr >= 1 && P.n_pt >= 0 && P.n_obs >= 0 &&
                    P.pt_offsets && (P.n_obs == 0 || (P.obs_img && P.obs_uv)) && P.img_intr,
                SFM_ERR_INVALID_ARG, "incomplete BA problem");
    SFM_REQUIRE(P.pt_offsets[0] == 0 && P.pt_offsets[P.n_pt] == P.n_obs, SFM_ERR_INVALID_ARG,
                "pt_offsets must run from 0 to n_obs");
    SFM_REQUIRE(P.n_obs < INT32_MAX && P.n_pt < INT32_MAX, SFM_ERR_UNSUPPORTED,
                "more than 2^31 observations per process");
    {
        // first offending point / observation per host range, reported in order
        std::vector<int64_t> bad_p(16, -1), bad_o(16, -1);
        parallel_ranges(P.n_pt, [&](int64_t p0, int64_t p1, int t) {
            for (int64_t p = p0; p < p1 && bad_p[t] < 0; ++p)
                if (P.pt_offsets[p + 1] < P.pt_offsets[p]) bad_p[t] = p;
        });
        parallel_ranges(P.n_obs, [&](int64_t o0, int64_t o1, int t) {
            for (int64_t o = o0; o < o1 && bad_o[t] < 0; ++o)
                if (P.obs_img[o] < 0 || P.obs_img[o] >= P.n_img) bad_o[t] = o;
        });
        for (int64_t p : bad_p)
            SFM_REQUIRE(p < 0, SFM_ERR_INVALID_ARG, "pt_offsets not monotone at point %lld", (long long)p);
        for (int64_t o : bad_o)
            SFM_REQUIRE(o < 0, SFM_ERR_INVALID_ARG, "obs %lld references image %d", (long long)o, P.obs_img[o]);
    }
    for (int i = 0; i < P.n_img; ++i)
        SFM_REQUIRE(P.img_intr[i] >= 0 && P.img_intr[i] < P.n_intr, SFM_ERR_INVALID_ARG,
                    "image %d references intrinsics %d", i, P.img_intr[i]);
    SFM_REQUIRE(P.const_img >= -1 && P.const_img < P.n_img, SFM_ERR_INVALID_ARG, "bad const_img");
    SFM_REQUIRE(sfm_ba_intr_width(P.camera_model) > 0, SFM_ERR_INVALID_ARG, "unknown camera_model %d",
                P.camera_model);
}

// RCS storage and solver, identical on every rank: the block-banded form
// (block cyclic reduction, ba_bcr.hip) for a camera band of <= 10 blocks
// and a few intrinsics blocks, else dense (blocked Cholesky, ba_dense.hip)
// (the band solver's arrow holds 4-wide intrinsics blocks: RADIAL3 is dense)
// (the BCR arrow carries iw * nintr <= 16 bordered columns: one MFMA column
// tile besides the rhs, and a corner system of at most 16 x 16)
void decide_rcs(BAHostPlan& pl, const PlanOpts& opts) {
    pl.dense = !(pl.D <= kBandMaxD && pl.iw * pl.nintr <= 16) || opts.force_dense;
    pl.n_sdense = 0;
    if (pl.dense) {
        SFM_REQUIRE(pl.nF <= 40000, SFM_ERR_UNSUPPORTED, "dense reduced camera system of %lld columns",
                    (long long)pl.nF);
        pl.n_sdense = pl.nF * pl.nF;
    }
}

// ---- Schur chunks ---------------------------------------------------------------
// Greedy over shard chunk points: a chunk's F blocks (camera 6 rows, intrinsics 4
// rows) must fit `cap` rows of its tile: 64 (4x4 MFMA tiles, -Zw on the
// VALU) or 76 (5x5 tiles, -Zw in row 79).  The 64-row form does 2/3 of the
// MFMA work per point; it is used unless it would need many more chunks.
// 128 points per chunk: ~2x the co-resident waves of the chip at C4 size,
// so the last round of chunks is short (256 measured 17% slower).
// A shard too small to give every wave slot of the chip a 128-point chunk
// (a landmark shard at N = 2, 4, 8) gets shorter chunks instead, down to 16
// points: the Schur pass takes about one chunk's latency once the chunks
// fit in one round of the chip's 2048 wave slots (256 CUs x 2 waves per
// SIMD x 4), and a chunk count just past a round costs a second one.  So
// the target is 1850 chunks, a margin for the camera-window cuts
// (profiles/r04/o_n8knobs/pts.txt, rank 0 of a C4 shard: N = 8 2147-2180
// LM-iters/s at 31 points (2107 chunks), 2272-2282 at 40; N = 4 1838-1870
// at 61, 1971-1981 at 75; N = 2 1427-1429 at 122, 1583-1592 at 128.
// Round 5, profiles/r05/w_tc*: target 1600 / 1750 / 1850 gives N = 4
// 2407 / 2431 / 2463 and N = 8 2958-2967 / 2920 / 2979 LM-iters/s (1619 /
// 1806 / 1870 chunks at N = 8, 1987 at N = 4 with 1850); fewer, longer
// chunks (872 / 998) leave SIMDs with one wave: N = 8 2651-2726).
#ifndef SFM_TARGET_CHUNKS
#define SFM_TARGET_CHUNKS 1850   // (A/B builds only)
#endif
constexpr int64_t kTargetChunks = SFM_TARGET_CHUNKS;
int chunk_pts_for(int64_t n_cpt) {
    return (int)std::max<int64_t>(16, std::min<int64_t>(kChunkPts, (n_cpt + kTargetChunks - 1) / kTargetChunks));
}
// Chunk points are chunked in fixed-length ranges on host threads (a chunk
// never spans two ranges): up to 65536 chunk points, ranges of 1024 (at most
// 63 extra chunks, against the ~1850 such a shard gets); above, 4096 points
// doubled until there are at most 16 ranges (at most 15 extra chunks out of
// thousands).  The ranges depend on the number of chunk points only, so a
// grown problem's chunking keeps every whole range before its first moved
// point and re-chunks about one range more than the growth moved (round 6;
// until round 5 the shard was cut into up to 16 equal parts).
int64_t chunk_range_len(int64_t ncp) {
    if (ncp <= 64 * 1024) return 1024;
    int64_t r = 4096;
    while (ncp > 16 * r) r *= 2;
    return r;
}
// algorithmic flops: the symmetric Z Z' over the point's own F
// rows (r(r+1)/2 entries x 3 x 2 = 3 r (r+1)), the linearisation (600 per
// observation) and the point block (V, its factor, M = Jx L^-T, Z = J' M: 180
// per observation + 30)
int64_t point_flops(int64_t rows, int64_t nobs) { return 3 * rows * (rows + 1) + 780 * nobs + 30; }

// resize an array a grown plan took over from its seed, with room for the
// next calls' growth (a reallocation copies the whole array)
template <class V>
void grow_to(V& v, size_t n) {
    if (v.capacity() < n) v.reserve(n + n / 4);
    v.resize(n);
}

// A chunking is abandoned as soon as its chunk count (over all ranges)
// passes abort_at: from there on its outcome no longer matters (see the
// choice of the tile height below), e.g. under random visibility, where
// chunks are dropped whatever the count.  The ranges add their chunks to
// one shared counter as they close them.
struct ChunkShared {
    std::atomic<int64_t> n_closed{0};
    std::atomic<bool> abandoned{false};
    int64_t abort_at = INT64_MAX;
};

// greedy chunking of shard chunk points [k_begin, k_end) at `cap` tile rows;
// slot_out is indexed by shard observation (each range writes its own)
int64_t chunk_range(const sfm_ba_problem& P, const BAHostPlan& pl, int cap, int chunk_pts, int group_pts,
                    int32_t k_begin, int32_t k_end, std::vector<ChunkDesc>& chunks_out, int32_t* slot_out,
                    ChunkShared& sh) {
    int64_t flops = 0;
    ChunkDesc cd{};
    std::vector<int> cams, intrs, dcams;  // F-slot images / intrinsics, staged images
    // O(1) membership for the open chunk: image -> F slot / staged index,
    // intrinsics -> staged index (-1 = absent); reset through the lists
    std::vector<int> cam_slot(P.n_img, -1), dcam_idx(P.n_img, -1), intr_idx(P.n_intr, -1);
    int rows = 0;
    auto reset = [&](int32_t p) {
        cd = ChunkDesc{};
        cd.pt_begin = p;
        cd.obs_begin = pl.pt_off[p];
        for (int s = 0; s < kMaxSlots; ++s) { cd.slot_img[s] = -1; cd.slot_intr[s] = -1; cd.slot_row[s] = -1; cd.slot_col[s] = -1; }
        for (int s = 0; s < kCamSlots; ++s) { cd.cam_img[s] = -1; cd.cam_row[s] = -1; cd.cam_col[s] = -1; }
        for (int s = 0; s < kIntrSlots; ++s) { cd.intr_id[s] = -1; cd.intr_row[s] = -1; cd.intr_col[s] = -1; }
        for (int img : cams) cam_slot[img] = -1;
        for (int img : dcams) dcam_idx[img] = -1;
        for (int q : intrs) intr_idx[q] = -1;
        cams.clear(); intrs.clear(); dcams.clear(); rows = 0;
    };
    // a tile group: its points split evenly into <= kGroupChunks chunks of
    // <= chunk_pts points, every chunk carrying the group's slot layout
    auto close = [&](int32_t p_end) {
        cd.pt_end = p_end;
        cd.obs_end = pl.pt_off[p_end];
        cd.n_slots = (int32_t)(cams.size() + intrs.size());
        cd.n_cams = (int32_t)dcams.size();
        cd.n_intr = (int32_t)intrs.size();
        const int32_t p0 = cd.pt_begin, npg = p_end - p0;
        const int n_sub = std::max(1, (npg + chunk_pts - 1) / chunk_pts);
        for (int j = 0; j < n_sub; ++j) {
            ChunkDesc sub = cd;
            sub.pt_begin = p0 + (int32_t)((int64_t)npg * j / n_sub);
            sub.pt_end = p0 + (int32_t)((int64_t)npg * (j + 1) / n_sub);
            sub.obs_begin = pl.pt_off[sub.pt_begin];
            sub.obs_end = pl.pt_off[sub.pt_end];
            sub.sub = j;
            chunks_out.push_back(sub);
        }
        if (sh.n_closed.fetch_add(n_sub, std::memory_order_relaxed) + n_sub > sh.abort_at)
            sh.abandoned.store(true, std::memory_order_relaxed);
    };
    // per-point image lists in fixed storage (<= kSubObs each): this loop
    // runs once per point, and heap vectors here dominated planning time
    struct Small {
        int v[kSubObs];
        int n = 0;
        void push_back(int x) { v[n++] = x; }
        const int* begin() const { return v; }
        const int* end() const { return v + n; }
        size_t size() const { return (size_t)n; }
        bool has(int x) const { return std::find(v, v + n, x) != v + n; }
    };
    if (k_end > k_begin) reset(k_begin);
    for (int32_t k = k_begin; k < k_end; ++k) {
        if (((k - k_begin) & 255) == 0 && sh.abandoned.load(std::memory_order_relaxed)) return flops;
        const int32_t nobs = pl.pt_off[k + 1] - pl.pt_off[k];
        Small pc, pi, pd;
        for (int32_t s = pl.pt_off[k]; s < pl.pt_off[k + 1]; ++s) {
            const int img = pl.obs_img[s];
            if (pl.cam_blk[img] >= 0) pc.push_back(img);
            pd.push_back(img);
            const int q = P.img_intr[img];
            if (!pi.has(q)) pi.push_back(q);
        }
        const int own = 6 * (int)pc.size() + pl.iw * (int)pi.size();
        SFM_REQUIRE(own <= cap, SFM_ERR_INVALID_ARG, "internal: chunk point over %d rows", cap);
        int add = 0, add_slots = 0, add_d = 0, add_i = 0;
        for (int img : pc) if (cam_slot[img] < 0) { add += 6; ++add_slots; }
        for (int q : pi) if (intr_idx[q] < 0) { add += pl.iw; ++add_slots; ++add_i; }
        for (int img : pd) if (dcam_idx[img] < 0) ++add_d;
        const bool full = k > cd.pt_begin &&
                          (rows + add > cap || k - cd.pt_begin >= group_pts ||
                           (int)(cams.size() + intrs.size()) + add_slots > kMaxSlots ||
                           (int)dcams.size() + add_d > kCamSlots ||
                           (int)intrs.size() + add_i > kIntrSlots);
        if (full) { close(k); reset(k); }
        for (int img : pc)
            if (cam_slot[img] < 0) {
                const int s = (int)(cams.size() + intrs.size());
                cams.push_back(img);
                cam_slot[img] = s;
                cd.slot_img[s] = img; cd.slot_row[s] = rows; cd.slot_col[s] = pl.img_colc[img];
                rows += 6;
            }
        for (int q : pi)
            if (intr_idx[q] < 0) {
                const int s = (int)(cams.size() + intrs.size());
                const int t = (int)intrs.size();
                intrs.push_back(q);
                intr_idx[q] = t;
                cd.slot_intr[s] = q; cd.slot_row[s] = rows;
                cd.slot_col[s] = (int32_t)(pl.nb + (int64_t)pl.iw * pl.intr_blk[q]);
                cd.intr_id[t] = q; cd.intr_row[t] = rows; cd.intr_col[t] = cd.slot_col[s];
                rows += pl.iw;
            }
        for (int img : pd)
            if (dcam_idx[img] < 0) {
                const int t = (int)dcams.size();
                dcams.push_back(img);
                dcam_idx[img] = t;
                cd.cam_img[t] = img;
                const int s = cam_slot[img];   // constant images have no F slot
                if (s >= 0) { cd.cam_row[t] = cd.slot_row[s]; cd.cam_col[t] = cd.slot_col[s]; }
            }
        // observation -> staged camera | staged intrinsics << 8
        for (int32_t s = pl.pt_off[k]; s < pl.pt_off[k + 1]; ++s) {
            const int img = pl.obs_img[s];
            slot_out[s] = dcam_idx[img] | (intr_idx[P.img_intr[img]] << 8);
        }
        flops += point_flops(own, nobs);
    }
    if (k_end > k_begin) close(k_end);
    return flops;
}

// One chunking at `cap` rows over the ranges [g_begin, nseg) of the chunk
// points [0, ncp) (the ranges before g_begin are a seed plan's, with
// `prefix_chunks` chunks).  Returns false if the chunking was abandoned (more
// than `limit` chunks in all).
struct Chunking {
    std::vector<std::vector<ChunkDesc>> seg;   // per range ([g_begin, nseg) filled)
    std::vector<int64_t> flops;
};
bool make_chunks(const sfm_ba_problem& P, const BAHostPlan& pl, int cap, int chunk_pts, int64_t rlen, int64_t ncp,
                 int g_begin, int64_t prefix_chunks, int64_t limit, Chunking& out, int32_t* slot_out) {
    const int nseg = (int)((ncp + rlen - 1) / rlen);
    out.seg.assign(nseg, {});
    out.flops.assign(nseg, 0);
    ChunkShared sh;
    sh.n_closed = prefix_chunks;
    sh.abort_at = limit;
    if (prefix_chunks > limit) return false;
    const int group_pts = schur_group(cap == 64 ? 4 : 5) * chunk_pts;
    std::vector<int> rc(nseg, SFM_OK);
    if (nseg > g_begin)
        parallel_segments(nseg - g_begin, [&](int q) {
            const int g = g_begin + q;
            rc[g] = guarded([&] {
                const int32_t k0 = (int32_t)(g * rlen), k1 = (int32_t)std::min<int64_t>(ncp, (g + 1) * rlen);
                out.flops[g] = chunk_range(P, pl, cap, chunk_pts, group_pts, k0, k1, out.seg[g], slot_out, sh);
                return SFM_OK;
            });
        });
    for (int g = 0; g < nseg; ++g)
        if (rc[g] != SFM_OK) throw SfmError{rc[g]};
    return !sh.abandoned.load();
}

// Per chunking range: the largest tile rows (6 per active camera, iw per
// intrinsics block) and observation count of one of its points
void range_shapes(const sfm_ba_problem& P, const BAHostPlan& pl, int64_t ncp, int64_t rlen, int g_begin,
                  std::vector<int32_t>& own, std::vector<int32_t>& obs) {
    const int nseg = (int)((ncp + rlen - 1) / rlen);
    own.resize(nseg);
    obs.resize(nseg);
    if (nseg > g_begin)
        parallel_segments(nseg - g_begin, [&](int q) {
            const int g = g_begin + q;
            int lo_own = 0, lo_obs = 0;
            const int64_t k1 = std::min<int64_t>(ncp, (g + 1) * rlen);
            for (int64_t k = g * rlen; k < k1; ++k) {
                lo_obs = std::max(lo_obs, pl.pt_off[k + 1] - pl.pt_off[k]);
                int nc = 0;
                int32_t pi[kIntrSlots];
                int ni = 0;
                for (int32_t s = pl.pt_off[k]; s < pl.pt_off[k + 1]; ++s) {
                    if (pl.cam_blk[pl.obs_img[s]] >= 0) ++nc;
                    const int q2 = P.img_intr[pl.obs_img[s]];
                    if (std::find(pi, pi + ni, q2) == pi + ni) pi[ni++] = q2;
                }
                lo_own = std::max(lo_own, 6 * nc + pl.iw * ni);
            }
            own[g] = lo_own;
            obs[g] = lo_obs;
        });
}

// What a grown plan takes from its seed (build_plan_grown)
struct Seed {
    BAHostPlan* q;
    int64_t pos0;   // the first sorted position the growth changes
};

// Shard arrays, Schur chunks and general points of a planned order (pl.order,
// pl.bounds).  With a seed, the sorted positions before seed->pos0 are the
// seed plan's (same points, same observations) and only what follows them is
// planned; every array ends up as the fresh plan makes it.
void plan_points(const sfm_ba_problem& P, BAHostPlan& pl, const PlanOpts& opts, Seed* sd, PhaseTimer& tm) {
    const int rank = pl.rank;
    const int64_t b0 = pl.bounds[rank], b1 = pl.bounds[rank + 1];
    BAHostPlan* q = sd ? sd->q : nullptr;
    const int64_t pos0 = sd ? sd->pos0 : 0;   // (world 1: shard positions = sorted positions)
    // ---- classification: chunkable points first, then general points --------
    std::vector<char> ck(b1 - b0);
    if (q) std::copy(q->grow.ck.begin(), q->grow.ck.begin() + pos0, ck.begin());
    parallel_ranges(b1 - b0 - pos0, [&](int64_t k0, int64_t k1, int) {
        for (int64_t k = pos0 + k0; k < pos0 + k1; ++k) ck[k] = chunkable(P, pl, pl.order[b0 + k]);
    });
    int64_t kc0 = 0;   // chunk points before pos0
    for (int64_t k = 0; k < pos0; ++k) kc0 += ck[k];
    const int64_t kg0 = pos0 - kc0;   // general points before pos0
    {
        std::vector<int64_t> gpts;
        pl.spt_global.clear();
        pl.spt_global.reserve(b1 - b0);
        for (int64_t k = b0; k < b1; ++k) {
            if (ck[k - b0]) pl.spt_global.push_back(pl.order[k]);
            else gpts.push_back(pl.order[k]);
        }
        pl.n_cpt = (int64_t)pl.spt_global.size();
        pl.spt_global.insert(pl.spt_global.end(), gpts.begin(), gpts.end());
    }
    const int64_t n_ck = pl.n_cpt;   // classified chunkable (the chunking may drop them)
    tm.mark("classify");
    pl.n_spt = b1 - b0;
    pl.pt_off.assign(pl.n_spt + 1, 0);
    for (int64_t k = 0; k < pl.n_spt; ++k) {
        const int64_t p = pl.spt_global[k];
        pl.pt_off[k + 1] = pl.pt_off[k] + (int32_t)(P.pt_offsets[p + 1] - P.pt_offsets[p]);
    }
    pl.n_sobs = pl.pt_off[pl.n_spt];
    tm.mark("pt_off");
    // the seed's general points before pos0 (observations in image order, their
    // slots and permutation): kept aside, their place moves with the chunk part
    std::vector<int32_t> gp_img, gp_slot, gp_perm;
    bool q_kept = false;
    if (q) {
        // the seed's general part = its non-chunkable points (it kept its chunks)
        q_kept = q->n_cpt == q->grow.n_ck;
        const int32_t qg0 = q->pt_off[q->n_cpt], qg1 = q->pt_off[q->n_cpt + kg0];
        if (q_kept && qg1 > qg0) {
            gp_img.assign(q->obs_img.begin() + qg0, q->obs_img.begin() + qg1);
            gp_slot.assign(q->obs_slot.begin() + qg0, q->obs_slot.begin() + qg1);
            if (!q->gobs_perm.empty()) {
                gp_perm.assign(q->gobs_perm.begin(), q->gobs_perm.begin() + (qg1 - qg0));
            } else {   // the seed's general points were all in image order
                gp_perm.resize(qg1 - qg0);
                for (int64_t g = 0; g < kg0; ++g) {
                    const int32_t s0 = q->pt_off[q->n_cpt + g] - qg0, s1 = q->pt_off[q->n_cpt + g + 1] - qg0;
                    for (int32_t s = s0; s < s1; ++s) gp_perm[s] = s - s0;
                }
            }
        }
        pl.obs_img = std::move(q->obs_img);
        pl.obs_slot = std::move(q->obs_slot);
    }
    // the chunk part before kc0 is the seed's, as it stands
    const int64_t s_keep = q ? pl.pt_off[kc0] : 0;
    grow_to(pl.obs_img, pl.n_sobs);
    if (!pl.uv_on_device) pl.obs_uv.resize(2 * pl.n_sobs);
    auto copy_obs = [&](int64_t k_lo, int64_t k_hi) {   // shard points [k_lo, k_hi) from the problem
        parallel_ranges(k_hi - k_lo, [&](int64_t a0, int64_t a1, int) {
            for (int64_t k = k_lo + a0; k < k_lo + a1; ++k) {
                const int64_t p = pl.spt_global[k];
                for (int64_t o = P.pt_offsets[p], s = pl.pt_off[k]; o < P.pt_offsets[p + 1]; ++o, ++s) {
                    pl.obs_img[s] = P.obs_img[o];
                    if (!pl.uv_on_device) {
                        pl.obs_uv[2 * s] = P.obs_uv[2 * o];
                        pl.obs_uv[2 * s + 1] = P.obs_uv[2 * o + 1];
                    }
                }
            }
        });
    };
    // fresh: every shard point; grown: the chunkable points from kc0 on (the
    // general part once the chunking has decided where it starts)
    if (q) copy_obs(kc0, n_ck);
    else copy_obs(0, pl.n_spt);
    (void)s_keep;
    tm.mark("shard");

    // ---- Schur chunks over [0, n_cpt) ------------------------------------------
    // Chunks of one tile group share one slot layout and one tile: the Schur
    // kernel runs a group as one workgroup, a wave per chunk, and adds the
    // waves' tiles in LDS (wave order) before the one write -- a quarter of the
    // tile traffic and of the reduce plan's tile terms of single-chunk tiles
    const int chunk_pts = chunk_pts_for(pl.n_cpt);
    const int64_t ncp = pl.n_cpt, rlen = chunk_range_len(ncp);
    const int nseg = (int)((ncp + rlen - 1) / rlen);
    // the seed's ranges before the one holding the first re-planned chunk point
    const bool same_ranges = q && q->grow.rlen == rlen;
    const int g_shape = same_ranges ? (int)(kc0 / rlen) : 0;
    std::vector<int32_t> seg_own, seg_obs;
    if (g_shape > 0) {
        seg_own.assign(q->grow.seg_own.begin(), q->grow.seg_own.begin() + g_shape);
        seg_obs.assign(q->grow.seg_obs.begin(), q->grow.seg_obs.begin() + g_shape);
    }
    range_shapes(P, pl, ncp, rlen, g_shape, seg_own, seg_obs);
    int max_own = 0, max_obs = 0;
    for (int g = 0; g < nseg; ++g) { max_own = std::max(max_own, seg_own[g]); max_obs = std::max(max_obs, seg_obs[g]); }
    tm.mark("chunk_shape");
    int64_t flops = 0;
    HostVec<int32_t> cslot;
    pl.tile_nt = 5;
    // Chunks pay off when camera windows are shared by many consecutive
    // points (sequences, orbits); under random visibility a chunk holds one
    // or two points and its tile traffic exceeds the general path's: a
    // chunking of more than n_cpt / 4 chunks is dropped
    const int64_t keep_max = pl.n_cpt / 4;
    bool kept = true;
    int kept_cap = 0;
    const bool both = max_own <= 64 && max_obs <= schur4_obs(P.camera_model) && !opts.tile80;
    std::vector<int32_t> seg_nch;
    std::vector<int64_t> seg_fl;
    auto take = [&](Chunking& c, int g_from) {   // ranges [g_from, nseg) of c after pl.chunks
        for (int g = g_from; g < nseg; ++g) {
            pl.chunks.insert(pl.chunks.end(), c.seg[g].begin(), c.seg[g].end());
            seg_nch.push_back((int32_t)c.seg[g].size());
            seg_fl.push_back(c.flops[g]);
        }
    };
    pl.chunks.clear();
    int64_t reused_chunks = 0;   // the seed's chunks at the head of pl.chunks
    // the 64-row kernel walks batches of at most schur4_obs observations
    if (both) {
        // both tile heights are planned (each over the host threads); the
        // 64-row one is taken unless it needs 5/4 as many chunks.  80 rows
        // over keep_max: dropped if taken, so 64 rows matter only within
        // keep_max; else 64 rows matter only within 5/4 of the 80-row count
        Chunking c4, c5;
        HostVec<int32_t> s4, s5;
        s4.resize(pl.pt_off[ncp]);
        s5.resize(pl.pt_off[ncp]);
        const bool ok5 = make_chunks(P, pl, kTileRowsUsed, chunk_pts, rlen, ncp, 0, 0, keep_max, c5, s5.data());
        int64_t n5 = 0;
        for (auto& v : c5.seg) n5 += (int64_t)v.size();
        const bool ok4 = make_chunks(P, pl, 64, chunk_pts, rlen, ncp, 0, 0, ok5 ? n5 * 5 / 4 : keep_max, c4, s4.data());
        if (ok4) {
            pl.tile_nt = 4; take(c4, 0); cslot.swap(s4); kept_cap = 64;
        } else if (ok5) {
            take(c5, 0); cslot.swap(s5); kept_cap = kTileRowsUsed;
        } else {
            kept = false;
        }
    } else {
        // one height: the seed's whole ranges before the first re-planned
        // chunk point are taken as they are (same chunk points, chunk length
        // and range length), the rest chunked
        const bool reuse = same_ranges && q_kept && q->grow.cap == kTileRowsUsed && q->grow.chunk_pts == chunk_pts;
        const int g0 = reuse ? (int)(kc0 / rlen) : 0;
        int64_t prefix = 0;
        if (reuse) {
            for (int g = 0; g < g0; ++g) prefix += q->grow.seg_nch[g];
            pl.chunks.assign(q->chunks.begin(), q->chunks.begin() + prefix);
            // the intrinsics' F columns follow the camera columns, whose count grew
            for (ChunkDesc& c : pl.chunks) {
                for (int a = 0; a < c.n_slots; ++a)
                    if (c.slot_intr[a] >= 0) c.slot_col[a] = (int32_t)(pl.nb + (int64_t)pl.iw * pl.intr_blk[c.slot_intr[a]]);
                for (int t = 0; t < c.n_intr; ++t)
                    c.intr_col[t] = (int32_t)(pl.nb + (int64_t)pl.iw * pl.intr_blk[c.intr_id[t]]);
            }
            seg_nch.assign(q->grow.seg_nch.begin(), q->grow.seg_nch.begin() + g0);
            seg_fl.assign(q->grow.seg_flops.begin(), q->grow.seg_flops.begin() + g0);
            cslot = std::move(pl.obs_slot);   // the seed's slots of those ranges, in place
            reused_chunks = prefix;
        }
        grow_to(cslot, pl.pt_off[ncp]);
        Chunking c5;
        kept = make_chunks(P, pl, kTileRowsUsed, chunk_pts, rlen, ncp, g0, prefix, keep_max, c5, cslot.data());
        if (kept) {
            take(c5, g0);
            kept_cap = kTileRowsUsed;
        }
    }
    for (int64_t f : seg_fl) flops += f;
    pl.reused_chunks = kept ? reused_chunks : 0;
    if (!kept || (pl.n_cpt > 0 && (int64_t)pl.chunks.size() * 4 > pl.n_cpt)) {
        pl.chunks.clear();
        cslot.clear();
        pl.n_cpt = 0;
        flops = 0;
        kept_cap = 0;
        seg_nch.clear();
        seg_fl.clear();
    }
    pl.group_off.clear();
    for (int32_t c = 0; c < (int32_t)pl.chunks.size(); ++c)
        if (pl.chunks[c].sub == 0) pl.group_off.push_back(c);
    pl.group_off.push_back((int32_t)pl.chunks.size());
    tm.mark("chunks");
    // the chunk points' slots are final; the general points' are written below
    grow_to(cslot, pl.n_sobs);
    pl.obs_slot.swap(cslot);
    pl.n_gpt = pl.n_spt - pl.n_cpt;

    // ---- general points ---------------------------------------------------------
    // (the seed's general points before pos0 are taken when both plans kept
    // their chunks: the same general points lead the same general part)
    const bool gen_reuse = q && q_kept && kept_cap != 0 && pl.n_cpt == n_ck;
    const int64_t gk0 = gen_reuse ? kg0 : 0;   // general points taken from the seed
    const int32_t gobs0 = pl.pt_off[pl.n_cpt];
    const int32_t gkeep = pl.pt_off[pl.n_cpt + gk0] - gobs0;   // their observations
    if (gen_reuse) {
        std::copy(gp_img.begin(), gp_img.begin() + gkeep, pl.obs_img.begin() + gobs0);
        std::copy(gp_slot.begin(), gp_slot.begin() + gkeep, pl.obs_slot.begin() + gobs0);
    }
    if (q) copy_obs(std::max<int64_t>(n_ck, pl.n_cpt + gk0), pl.n_spt);
    // a general point's observations in image order, so that repeated views
    // of one image are adjacent (the Z kernel sums runs of one camera block);
    // the permutation is kept for the plan cache's value refresh
    pl.gobs_perm.assign(pl.n_sobs - gobs0, 0);
    int permuted[16] = {0};
    if (gen_reuse && gkeep > 0) {
        std::copy(gp_perm.begin(), gp_perm.begin() + gkeep, pl.gobs_perm.begin());
        for (int64_t g = 0; g < gk0 && !permuted[0]; ++g) {
            const int32_t s0 = pl.pt_off[pl.n_cpt + g] - gobs0, s1 = pl.pt_off[pl.n_cpt + g + 1] - gobs0;
            for (int32_t s = s0; s < s1; ++s) permuted[0] |= pl.gobs_perm[s] != s - s0;
        }
    }
    parallel_ranges(pl.n_gpt - gk0, [&](int64_t a0, int64_t a1, int t) {
        std::vector<int32_t> idx;
        std::vector<int32_t> img;
        std::vector<double> uv;
        for (int64_t g = gk0 + a0; g < gk0 + a1; ++g) {
            const int64_t k = pl.n_cpt + g;
            const int32_t s0 = pl.pt_off[k], n = pl.pt_off[k + 1] - s0;
            idx.resize(n);
            std::iota(idx.begin(), idx.end(), 0);
            auto before = [&](int32_t a, int32_t b) { return pl.obs_img[s0 + a] < pl.obs_img[s0 + b]; };
            if (n <= 64) {   // insertion sort: stable, no buffer (stable_sort allocated one per point)
                for (int32_t r0 = 1; r0 < n; ++r0) {
                    const int32_t x = idx[r0];
                    int32_t r = r0;
                    for (; r > 0 && before(x, idx[r - 1]); --r) idx[r] = idx[r - 1];
                    idx[r] = x;
                }
            } else {
                std::stable_sort(idx.begin(), idx.end(), before);
            }
            bool moved = false;
            for (int32_t r = 0; r < n; ++r) moved |= idx[r] != r;
            if (moved) {
                img.assign(pl.obs_img.begin() + s0, pl.obs_img.begin() + s0 + n);
                for (int32_t r = 0; r < n; ++r) pl.obs_img[s0 + r] = img[idx[r]];
                if (!pl.uv_on_device) {
                    uv.assign(pl.obs_uv.begin() + 2 * s0, pl.obs_uv.begin() + 2 * (s0 + n));
                    for (int32_t r = 0; r < n; ++r) {
                        pl.obs_uv[2 * (s0 + r)] = uv[2 * idx[r]];
                        pl.obs_uv[2 * (s0 + r) + 1] = uv[2 * idx[r] + 1];
                    }
                }
                permuted[t] = 1;
            }
            for (int32_t r = 0; r < n; ++r) pl.gobs_perm[s0 + r - gobs0] = idx[r];
        }
    });
    if (std::none_of(permuted, permuted + 16, [](int v) { return v != 0; })) pl.gobs_perm.clear();

    // ---- general points: their F blocks and Z buffer layout --------------------
    // blocks in F-column order; obs_slot = local camera block (0xffff: constant
    // image) | local intrinsics block << 16
    std::vector<int64_t> gflops(pl.n_gpt, 0);
    if (gen_reuse) {
        pl.gblk_off = std::move(q->gblk_off);
        pl.gz_off = std::move(q->gz_off);
        pl.gblk_col = std::move(q->gblk_col);
        pl.gblk_z = std::move(q->gblk_z);
        std::copy(q->grow.gflops.begin(), q->grow.gflops.begin() + gk0, gflops.begin());
    }
    if (gen_reuse && pl.nb != q->nb) {   // the seed's intrinsics columns, moved behind the new cameras'
        const int32_t shift = (int32_t)(pl.nb - q->nb);
        for (int32_t a = 0; a < pl.gblk_off[gk0]; ++a)
            if (pl.gblk_col[a] >= q->nb) pl.gblk_col[a] += shift;
    }
    grow_to(pl.gblk_off, pl.n_gpt + 1);
    grow_to(pl.gz_off, pl.n_gpt + 1);
    pl.gblk_off[0] = 0;
    pl.gz_off[0] = 0;
    pl.gz_max = 0;
    {
        // two passes on the host threads: block counts and Z sizes per point,
        // then (after the prefix sums) every point writes its own blocks
        auto point_cols = [&](int64_t k, std::vector<int32_t>& cols) {
            cols.clear();
            for (int32_t s = pl.pt_off[k]; s < pl.pt_off[k + 1]; ++s) {
                const int img = pl.obs_img[s];
                if (pl.img_colc[img] >= 0) cols.push_back(pl.img_colc[img]);
                cols.push_back(pl.img_coli[img]);
            }
            std::sort(cols.begin(), cols.end());
            cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
        };
        auto zrows = [&](const std::vector<int32_t>& cols) {
            int32_t z = 0;
            for (int32_t c : cols) z += 3 * (c < pl.nb ? 6 : pl.iw);
            return z;
        };
        // per-point counts in [g + 1] (the seed's prefix sums stay for g < gk0)
        std::vector<int32_t> nblk(pl.n_gpt - gk0), nz(pl.n_gpt - gk0);
        parallel_ranges(pl.n_gpt - gk0, [&](int64_t a0, int64_t a1, int) {
            std::vector<int32_t> cols;
            for (int64_t a = a0; a < a1; ++a) {
                const int64_t g = gk0 + a, k = pl.n_cpt + g;
                point_cols(k, cols);
                SFM_REQUIRE(cols.size() < 0xffff, SFM_ERR_UNSUPPORTED, "point with %zu parameter blocks", cols.size());
                const int32_t z = zrows(cols);
                SFM_REQUIRE(z + 3 <= kZMaxDoubles, SFM_ERR_UNSUPPORTED,
                            "point %lld observed by %zu parameter blocks (more than the %d rows one wavefront eliminates)",
                            (long long)pl.spt_global[k], cols.size(), kZMaxDoubles / 3);
                nblk[a] = (int32_t)cols.size();
                nz[a] = z + 3;   // + w = L^-1 g_E
            }
        });
        for (int64_t g = 0; g < gk0; ++g) pl.gz_max = std::max<int64_t>(pl.gz_max, pl.gz_off[g + 1] - pl.gz_off[g]);
        for (int64_t g = gk0; g < pl.n_gpt; ++g) {
            pl.gz_max = std::max<int64_t>(pl.gz_max, nz[g - gk0]);
            pl.gblk_off[g + 1] = pl.gblk_off[g] + nblk[g - gk0];
            pl.gz_off[g + 1] = pl.gz_off[g] + nz[g - gk0];
        }
        grow_to(pl.gblk_col, pl.gblk_off[pl.n_gpt]);
        grow_to(pl.gblk_z, pl.gblk_off[pl.n_gpt]);
        parallel_ranges(pl.n_gpt - gk0, [&](int64_t a0, int64_t a1, int) {
            std::vector<int32_t> cols;
            for (int64_t g = gk0 + a0; g < gk0 + a1; ++g) {
                const int64_t k = pl.n_cpt + g;
                point_cols(k, cols);
                int32_t z = 0, qb = pl.gblk_off[g];
                for (int32_t c : cols) {
                    pl.gblk_col[qb] = c;
                    pl.gblk_z[qb++] = z;
                    z += 3 * (c < pl.nb ? 6 : pl.iw);
                }
                for (int32_t s = pl.pt_off[k]; s < pl.pt_off[k + 1]; ++s) {
                    const int img = pl.obs_img[s];
                    const int32_t cb = pl.img_colc[img] >= 0
                                           ? (int32_t)(std::lower_bound(cols.begin(), cols.end(), pl.img_colc[img]) - cols.begin())
                                           : 0xffff;
                    const int32_t ib = (int32_t)(std::lower_bound(cols.begin(), cols.end(), pl.img_coli[img]) - cols.begin());
                    pl.obs_slot[s] = cb | (ib << 16);
                }
                gflops[g] = point_flops(z / 3, pl.pt_off[k + 1] - pl.pt_off[k]);
            }
        });
        for (int64_t f : gflops) flops += f;
        pl.n_z = pl.gz_off[pl.n_gpt];
        SFM_REQUIRE(pl.n_z < INT32_MAX, SFM_ERR_UNSUPPORTED, "general points' Z buffer of %lld doubles",
                    (long long)pl.n_z);
        // Z kernel work: batches of consecutive short points, the rest alone
        pl.zbatch.clear();
        pl.zlong.clear();
        int32_t g0 = -1, nobs = 0;
        auto close = [&](int32_t g1) {
            if (g0 >= 0) { pl.zbatch.push_back(g0); pl.zbatch.push_back(g1); }
            g0 = -1;
            nobs = 0;
        };
        for (int32_t g = 0; g < (int32_t)pl.n_gpt; ++g) {
            const int64_t k = pl.n_cpt + g;
            const int32_t n = pl.pt_off[k + 1] - pl.pt_off[k];
            if (n > kZShortObs) {
                close(g);
                pl.zlong.push_back(g);
                continue;
            }
            if (g0 >= 0 && (nobs + n > 64 || g - g0 >= kZBatchPts)) close(g);
            if (g0 < 0) g0 = g;
            nobs += n;
        }
        close((int32_t)pl.n_gpt);
    }
    tm.mark("general");
    pl.reused_pts = pos0;
    pl.reused_gpts = gk0;
    if (pl.n_cpt == 0) pl.reused_chunks = 0;
    // what the next grown plan takes (world 1)
    PlanGrowState& gs = pl.grow;
    gs.ck = std::move(ck);
    gs.rlen = rlen;
    gs.chunk_pts = chunk_pts;
    gs.n_ck = n_ck;
    gs.cap = !both && kept_cap == kTileRowsUsed ? kept_cap : 0;   // (a two-height choice is re-planned)
    gs.seg_nch = std::move(seg_nch);
    gs.seg_flops = std::move(seg_fl);
    gs.seg_own = std::move(seg_own);
    gs.seg_obs = std::move(seg_obs);
    gs.gflops = std::move(gflops);
    // the observation arrays are final from here on: the caller may start
    // their upload while the reduce plan is built
    if (pl.on_shard_ready) pl.on_shard_ready(pl);
    tm.mark("shard_ready");
    pl.schur_flops = flops;
    pl.schur_bytes = pl.n_sobs * (16 + 4 + 4 + 4) + pl.n_spt * (24 + 24 + 4) +
                     (int64_t)pl.n_group() * kTileR * kTileR * 8;

    // ---- observations per image (the image-ordered copy itself is built on
    // the device from the uploaded shard arrays: ba_image_order) -------------
    pl.img_obs_ptr.assign(P.n_img + 1, 0);
    {
        constexpr int kMaxT = 16;
        std::vector<std::vector<int32_t>> cnt(kMaxT);
        parallel_ranges(pl.n_sobs, [&](int64_t s0, int64_t s1, int t) {
            cnt[t].assign(P.n_img, 0);
            for (int64_t s = s0; s < s1; ++s) cnt[t][pl.obs_img[s]]++;
        });
        for (int i = 0; i < P.n_img; ++i) {
            int32_t tot = 0;
            for (int t = 0; t < kMaxT; ++t)
                if (!cnt[t].empty()) tot += cnt[t][i];
            pl.img_obs_ptr[i + 1] = pl.img_obs_ptr[i] + tot;
        }
        // image Gram workgroups per image from the shard's observations per
        // image (profiles/r04/cc_gseg: C4 at N = 1, ~5000 each: 1086-1088 /
        // 1080-1083 / 1047-1052 LM-iters/s with 3 / 4 / 6; rank 0 of N = 8,
        // ~625 each: 2438-2444 / 2398-2401 / 2344-2347 with 2 / 3 / 4, and one
        // measured slower than three, profiles/r04/k_shard)
        pl.gram_img.clear();
        for (int i = 0; i < P.n_img; ++i)
            if (pl.img_obs_ptr[i + 1] != pl.img_obs_ptr[i]) pl.gram_img.push_back(i);
        const int64_t seen = (int64_t)pl.gram_img.size();
        const int64_t avg = seen > 0 ? pl.n_sobs / seen : 0;
        pl.gram_seg = std::min<int32_t>(kGramSeg, avg >= 1600 ? 3 : avg >= 128 ? 2 : 1);
    }
    tm.mark("image_csr");
}

void build_reduce_plan(const sfm_ba_problem& P, BAHostPlan& pl, PhaseTimer& tm, BAHostPlan* seed = nullptr);

}  // namespace

void build_plan(const sfm_ba_problem& P, int rank, int world, BAHostPlan& pl, const PlanOpts& opts) {
    validate_problem(P);
    PhaseTimer tm("build_plan");
    tm.mark("validate");
    pl.n_img = P.n_img; pl.n_intr = P.n_intr; pl.n_pt = P.n_pt; pl.n_obs = P.n_obs;
    pl.rank = rank; pl.world = world;
    PointSpans spans;   // every point's active camera span: the partition's sort keys
    std::vector<char> im;   // observed images
    bool rcm = false;
    int32_t lb = 0;
    pl.cam_blk = camera_blocks(P, &pl.ncam, &pl.D, &spans, &im, &lb, &rcm);
    active_from_blocks(P, pl, im);
    tm.mark("active");
    decide_rcs(pl, opts);
    partition_points(P, pl.cam_blk, world, pl.order, pl.bounds, &spans);
    tm.mark("partition");
    plan_points(P, pl, opts, nullptr, tm);
    build_reduce_plan(P, pl, tm);
    // a grown problem's plan can start from this one (world 1, the images'
    // own camera order: a reordering moves every camera)
    PlanGrowState& gs = pl.grow;
    gs.ok = world == 1 && !rcm;
    if (gs.ok) {
        gs.span_lo = std::move(spans.lo);
        gs.span_hi = std::move(spans.hi);
        gs.used = std::move(im);
        gs.lb = lb;
    }
}

bool build_plan_grown(const sfm_ba_problem& P, const GrowPrev& prev, BAHostPlan& q, BAHostPlan& pl,
                      const PlanOpts& opts) {
    // ---- does P grow prev, and can q seed it?  (nothing of q moves before
    // every check has passed) ----------------------------------------------------
    if (!q.grow.ok || q.world != 1 || q.n_pt != prev.n_pt || q.n_obs != prev.n_obs || q.n_img != prev.n_img) return false;
    if (P.n_intr != prev.n_intr || P.const_img != prev.const_img || P.camera_model != prev.model ||
        P.n_img < prev.n_img || P.n_pt < prev.n_pt || P.n_obs < prev.n_obs || !P.pt_offsets || !P.img_intr ||
        (P.n_obs > 0 && !P.obs_img))
        return false;
    if (prev.n_img > 0 && std::memcmp(P.img_intr, prev.img_intr, sizeof(int32_t) * prev.n_img) != 0) return false;
    validate_problem(P);
    PhaseTimer tm("build_plan_grown");
    const int64_t n_old = prev.n_pt;
    // every old point keeps its observations, in order, and may gain new ones
    std::vector<char> chg(n_old, 0);
    {
        int bad[16] = {0};
        parallel_ranges(n_old, [&](int64_t p0, int64_t p1, int t) {
            for (int64_t p = p0; p < p1 && !bad[t]; ++p) {
                const int64_t n0 = prev.pt_offsets[p + 1] - prev.pt_offsets[p], n1 = P.pt_offsets[p + 1] - P.pt_offsets[p];
                if (n1 < n0 || std::memcmp(P.obs_img + P.pt_offsets[p], prev.obs_img + prev.pt_offsets[p],
                                           sizeof(int32_t) * n0) != 0)
                    bad[t] = 1;
                chg[p] = n1 != n0;
            }
        });
        if (std::any_of(bad, bad + 16, [](int v) { return v != 0; })) return false;
    }
    tm.mark("check");
    // observed images and camera blocks: the old images keep their blocks
    std::vector<char> used(q.grow.used);
    used.resize(P.n_img, 0);
    auto each_new_obs = [&](auto&& fn) {   // observations appended to old points, then the new points'
        for (int64_t p = 0; p < n_old; ++p)
            if (chg[p])
                for (int64_t o = P.pt_offsets[p] + (prev.pt_offsets[p + 1] - prev.pt_offsets[p]); o < P.pt_offsets[p + 1]; ++o)
                    fn(o);
        for (int64_t o = P.pt_offsets[n_old]; o < P.n_obs; ++o) fn(o);
    };
    each_new_obs([&](int64_t o) { used[P.obs_img[o]] = 1; });
    std::vector<int32_t> cam_blk(P.n_img, -1);
    int32_t ncam = 0;
    for (int i = 0; i < P.n_img; ++i)
        if (used[i] && i != P.const_img) cam_blk[i] = ncam++;
    for (int i = 0; i < prev.n_img; ++i)
        if (cam_blk[i] != q.cam_blk[i]) return false;
    {   // the same active intrinsics blocks
        std::vector<char> iu(P.n_intr, 0);
        for (int i = 0; i < P.n_img; ++i)
            if (used[i]) iu[P.img_intr[i]] = 1;
        for (int k = 0; k < P.n_intr; ++k)
            if ((iu[k] != 0) != (q.intr_blk[k] >= 0)) return false;
    }
    // spans, the half bandwidth and the long-track bound of the moved points
    std::vector<int32_t> lo(q.grow.span_lo), hi(q.grow.span_hi);
    lo.resize(P.n_pt);
    hi.resize(P.n_pt);
    int32_t D = q.D, lb = q.grow.lb;
    std::vector<int64_t> moved;   // old points with new observations, then the new points
    for (int64_t p = 0; p < n_old; ++p)
        if (chg[p]) moved.push_back(p);
    for (int64_t p = n_old; p < P.n_pt; ++p) moved.push_back(p);
    {
        std::vector<int32_t> cs;
        for (int64_t p : moved) {
            int l = INT_MAX, h = -1;
            cs.clear();
            for (int64_t o = P.pt_offsets[p]; o < P.pt_offsets[p + 1]; ++o) {
                const int b = cam_blk[P.obs_img[o]];
                if (b >= 0) { l = std::min(l, b); h = std::max(h, b); cs.push_back(b); }
            }
            if (h >= 0) D = std::max(D, h - l);
            lo[p] = h >= 0 ? l : ncam;
            hi[p] = h + 1;
            std::sort(cs.begin(), cs.end());
            lb = std::max(lb, (int32_t)(std::unique(cs.begin(), cs.end()) - cs.begin()) - 1);
        }
    }
    // the unmoved points without an active camera sort last: their key (ncam, 0)
    // moves with ncam
    if (ncam != q.ncam)
        for (int64_t p = 0; p < n_old; ++p)
            if (!chg[p] && hi[p] == 0) return false;
    // build_plan would try a reverse Cuthill-McKee order here (camera_blocks)
    if (D > kBandMaxD && lb <= kBandMaxD && ncam > 2 && P.n_obs <= (int64_t)8 << 20) return false;
    tm.mark("active");

    // ---- from here on q is consumed -------------------------------------------------
    pl.n_img = P.n_img; pl.n_intr = P.n_intr; pl.n_pt = P.n_pt; pl.n_obs = P.n_obs;
    pl.rank = 0; pl.world = 1;
    pl.uv_on_device = true;
    pl.cam_blk = std::move(cam_blk);
    pl.ncam = ncam;
    pl.D = D;
    active_from_blocks(P, pl, used);
    decide_rcs(pl, opts);
    // the sorted order: the unmoved points keep their relative order (their
    // keys did not change), the moved ones are merged in by (first, last
    // camera block, index) -- the order of build_plan's stable counting sorts
    auto less = [&](int64_t a, int64_t b) {
        return lo[a] != lo[b] ? lo[a] < lo[b] : hi[a] != hi[b] ? hi[a] < hi[b] : a < b;
    };
    std::sort(moved.begin(), moved.end(), less);
    pl.order.resize(P.n_pt);
    {
        size_t m = 0;
        int64_t k = 0;
        for (int64_t p : q.order) {
            if (chg[p]) continue;
            while (m < moved.size() && less(moved[m], p)) pl.order[k++] = moved[m++];
            pl.order[k++] = p;
        }
        while (m < moved.size()) pl.order[k++] = moved[m++];
    }
    // the first sorted position that differs, or holds a point with new
    // observations (a moved point may land where it was)
    int64_t pos0 = 0;
    while (pos0 < n_old && pl.order[pos0] == q.order[pos0] && !chg[pl.order[pos0]]) ++pos0;
    pl.bounds = {0, P.n_pt};
    tm.mark("order");
    Seed sd{&q, pos0};
    plan_points(P, pl, opts, &sd, tm);
    build_reduce_plan(P, pl, tm, &q);
    PlanGrowState& gs = pl.grow;
    gs.ok = true;
    gs.span_lo = std::move(lo);
    gs.span_hi = std::move(hi);
    gs.used = std::move(used);
    gs.lb = lb;
    q.grow.ok = false;   // (its arrays are partly moved)
    return true;
}

namespace {

void build_reduce_plan(const sfm_ba_problem& P, BAHostPlan& pl, PhaseTimer& tm, BAHostPlan* seed) {
    const int world = pl.world;
    // ---- reduce plan -----------------------------------------------------------
    // Every matrix block (a, b), a >= b in F-block order (cameras, then
    // intrinsics), is a target summing its terms in a fixed order: sum terms
    // (image Gram slices in image order, then chunk tile sub-blocks in tile
    // group order) and product terms (general points in order); vectors (rhs,
    // bF, cnF) likewise per block -- so every sum is bit-reproducible.  Both
    // lists are laid out target after target.  They are built by a counting
    // scatter over F-block rows, without materialising or sorting (key, term)
    // lists: per-row term counts first (one pass over the sources, O(blocks)),
    // which fix every row's first position; then each host thread takes a
    // range of rows, counts its targets' terms, and writes every term of its
    // rows straight to its final place, visiting the sources in their order.
    const int32_t nFB = pl.nFB, ncam = pl.ncam, nintr = pl.nintr, D = pl.D;
    const int Dp = D + 1;
    const bool band = !pl.dense;
    if (band) {
        pl.n_sband = (int64_t)ncam * Dp * 36;
        pl.n_sarrow = (int64_t)nintr * ncam * 6 * pl.iw;
        pl.n_scorner = (int64_t)nintr * nintr * pl.iw * pl.iw;
    }
    auto fb_of_col = [&](int64_t col) -> int32_t {
        return col < pl.nb ? (int32_t)(col / 6) : (int32_t)(ncam + (col - pl.nb) / pl.iw);
    };
    auto col_of_fb = [&](int32_t b) -> int64_t { return b < ncam ? 6LL * b : pl.nb + (int64_t)pl.iw * (b - ncam); };
    auto size_of_fb = [&](int32_t b) { return b < ncam ? 6 : pl.iw; };
    // Terms are stored resolved against the solver's one source buffer
    // [chunk tiles | U | Ub | Ucn] (ba_solver.cpp create_plan: the same layout)
    const int64_t fw = 6 + pl.iw;
    const int64_t o_u = std::max<int64_t>(pl.n_group(), 1) * kTileR * kTileR, o_ub = o_u + fw * fw * P.n_img * kGramSeg,
                  o_ucn = o_ub + fw * P.n_img * kGramSeg;
    auto flat = [&](const ReduceTerm& q, bool vec) {
        FlatTerm f{};
        f.sign = q.sign;
        f.mode = kFlatRows;
        switch (q.kind) {
            case kSrcTile: {
                // slot blocks occupy disjoint tile rows, so a block of two
                // slots is wholly below or wholly above the diagonal
                const int64_t base = (int64_t)q.index * kTileR * kTileR;
                if (vec || q.roff > q.coff) {
                    f.off = base + q.roff * kTileR + q.coff;
                    f.rs = vec ? 1 : kTileR;
                } else if (q.roff < q.coff) {
                    f.off = base + q.coff * kTileR + q.roff;
                    f.rs = 1;
                    f.mode = kFlatTrans;
                } else {   // rs = the origin's offset within the tile
                    f.off = base + q.roff * kTileR + q.coff;
                    f.rs = (int16_t)(q.roff * kTileR + q.coff);
                    f.mode = kFlatSym;
                }
                break;
            }
            case kSrcU:
                f.off = o_u + q.index * fw * fw + q.roff * fw + q.coff;
                f.rs = (int16_t)fw;
                break;
            case kSrcUb:
                f.off = o_ub + q.index * fw + q.roff;
                f.rs = 1;
                break;
            default:
                f.off = o_ucn + q.index * fw + q.roff;
                f.rs = 1;
                break;
        }
        return f;
    };
    // band: a corner block (k, l), k < l, is stored too, as the transpose of
    // (l, k): terms of an off-diagonal corner key go to two targets
    auto twice = [&](int32_t fa, int32_t fb) { return band && fb >= ncam && fb != fa; };
    // a tile group's window can be wider than the band: its slot pairs
    // further apart than D are structurally zero (no point sees both) and
    // have no target
    auto held = [&](int32_t fa, int32_t fb) { return !band || fa >= ncam || fa - fb <= D; };
    // the images that contribute Gram slices: (image, camera block, F block of its intrinsics)
    struct ImgSrc {
        int32_t img, cb, fq;
    };
    std::vector<ImgSrc> isrc;
    for (int img = 0; img < P.n_img; ++img) {
        const int cb = pl.cam_blk[img], q = pl.intr_blk[P.img_intr[img]];
        const bool seen = pl.img_obs_ptr[img + 1] != pl.img_obs_ptr[img];
        if (!seen && cb < 0 && q < 0) continue;
        // a landmark shard: an image none of this rank's observations sees
        // contributes nothing here (its blocks come from the other ranks)
        if (world > 1 && !seen) continue;
        isrc.push_back({img, cb, q >= 0 ? ncam + q : -1});
    }
    const int32_t ngrp = (int32_t)pl.n_group();
    auto grp = [&](int32_t c) -> const ChunkDesc& { return pl.chunks[pl.group_off[c]]; };
    // F-block range of every tile group and general point (rows they write)
    std::vector<int32_t> g_lo(ngrp), g_hi(ngrp), p_lo(pl.n_gpt), p_hi(pl.n_gpt);
    // F block of every general-point block (pfb) and tile-group slot (gfb)
    std::vector<int32_t> pfb(pl.gblk_col.size()), gfb((size_t)ngrp * kMaxSlots);
    for (int32_t c = 0; c < ngrp; ++c) {
        int32_t lo = INT32_MAX, hi = -1;
        for (int a = 0; a < grp(c).n_slots; ++a) {
            const int32_t f = fb_of_col(grp(c).slot_col[a]);
            gfb[(size_t)c * kMaxSlots + a] = f;
            lo = std::min(lo, f);
            hi = std::max(hi, f);
        }
        g_lo[c] = lo;
        g_hi[c] = hi;
    }
    parallel_ranges(pl.n_gpt, [&](int64_t g0, int64_t g1, int) {
        for (int64_t g = g0; g < g1; ++g) {
            const int32_t k0 = pl.gblk_off[g], k1 = pl.gblk_off[g + 1];
            for (int32_t a = k0; a < k1; ++a) pfb[a] = fb_of_col(pl.gblk_col[a]);
            p_lo[g] = k1 > k0 ? fb_of_col(pl.gblk_col[k0]) : INT32_MAX;   // columns ascend
            p_hi[g] = k1 > k0 ? fb_of_col(pl.gblk_col[k1 - 1]) : -1;
        }
    });
    tm.mark("terms_sources");

    // ---- per-row counts: matrix sum / product terms, rhs sum / product
    // terms, image slices (bF and cnF) ------------------------------------------
    enum { kMc, kMp, kVc, kVp, kVb, kNC };
    std::vector<int64_t> rc((size_t)kNC * (nFB + 1), 0);
    auto RC = [&](int w, int32_t f) -> int64_t& { return rc[(size_t)w * (nFB + 1) + f]; };
    const int32_t gseg = pl.gram_seg;
    for (const ImgSrc& s : isrc) {
        if (s.cb >= 0) {
            RC(kMc, s.cb) += gseg;
            if (s.fq >= 0) RC(kMc, s.fq) += gseg;
            RC(kVc, s.cb) += gseg;
            RC(kVb, s.cb) += gseg;
        }
        if (s.fq >= 0) {
            RC(kMc, s.fq) += gseg;
            RC(kVc, s.fq) += gseg;
            RC(kVb, s.fq) += gseg;
        }
    }
    {
        // tile groups and general points, per host range into private rows
        std::vector<std::vector<int64_t>> part(16);
        auto acc_groups = [&](int64_t c0, int64_t c1, std::vector<int64_t>& r) {
            for (int64_t c = c0; c < c1; ++c) {
                const ChunkDesc& cd = grp((int32_t)c);
                for (int a = 0; a < cd.n_slots; ++a) {
                    const int32_t fa = gfb[(size_t)c * kMaxSlots + a];
                    r[(size_t)kVc * (nFB + 1) + fa] += 1;
                    for (int b = 0; b < cd.n_slots; ++b) {
                        const int32_t fb = gfb[(size_t)c * kMaxSlots + b];
                        if (fa >= fb && held(fa, fb)) r[(size_t)kMc * (nFB + 1) + fa] += twice(fa, fb) ? 2 : 1;
                    }
                }
            }
        };
        auto acc_points = [&](int64_t g0, int64_t g1, std::vector<int64_t>& r) {
            for (int64_t g = g0; g < g1; ++g) {
                const int32_t k0 = pl.gblk_off[g], k1 = pl.gblk_off[g + 1];
                int32_t first_i = k1;   // first intrinsics block (columns ascend)
                for (int32_t a = k0; a < k1; ++a) {
                    const int32_t fa = pfb[a];
                    if (fa >= ncam && first_i == k1) first_i = a;
                    r[(size_t)kVp * (nFB + 1) + fa] += 1;
                    const int64_t pairs = a - k0 + 1, dbl = band && fa >= ncam ? a - first_i : 0;
                    r[(size_t)kMp * (nFB + 1) + fa] += pairs + dbl;
                }
            }
        };
        parallel_ranges(ngrp, [&](int64_t c0, int64_t c1, int t) {
            part[t].assign((size_t)kNC * (nFB + 1), 0);
            acc_groups(c0, c1, part[t]);
        });
        for (auto& p : part) {
            if (p.empty()) continue;
            for (size_t k = 0; k < p.size(); ++k) rc[k] += p[k];
            p.clear();
        }
        parallel_ranges(pl.n_gpt, [&](int64_t g0, int64_t g1, int t) {
            part[t].assign((size_t)kNC * (nFB + 1), 0);
            acc_points(g0, g1, part[t]);
        });
        for (auto& p : part)
            for (size_t k = 0; k < p.size(); ++k) rc[k] += p[k];
    }
    // first position of every row in its list: matrix sum terms, then rhs,
    // bF and cnF sum terms; matrix product terms, then rhs product terms
    std::vector<int64_t> base((size_t)kNC * (nFB + 1) + 1, 0);
    auto BS = [&](int w, int32_t f) -> int64_t& { return base[(size_t)w * (nFB + 1) + f]; };
    int64_t n_mc = 0, n_mp = 0, n_vc = 0, n_vp = 0, n_vb = 0;
    for (int32_t f = 0; f < nFB; ++f) {
        BS(kMc, f) = n_mc; n_mc += RC(kMc, f);
        BS(kMp, f) = n_mp; n_mp += RC(kMp, f);
        BS(kVc, f) = n_vc; n_vc += RC(kVc, f);
        BS(kVp, f) = n_vp; n_vp += RC(kVp, f);
        BS(kVb, f) = n_vb; n_vb += RC(kVb, f);
    }
    BS(kMc, nFB) = n_mc; BS(kMp, nFB) = n_mp;
    const int64_t n_terms = n_mc + n_vc + 2 * n_vb, n_pterms = n_mp + n_vp;
    SFM_REQUIRE(n_terms < INT32_MAX && n_pterms < INT32_MAX, SFM_ERR_UNSUPPORTED,
                "reduce plan of %lld sum / %lld product terms", (long long)n_terms, (long long)n_pterms);
    // A grown plan (seed): the matrix rows before f0 -- the first F-block row
    // a re-planned chunk or general point writes, or a new camera's -- are the
    // seed's, targets and terms alike (the same sources in the same order), in
    // place; only their image-slice offsets (behind the tiles in the source
    // buffer, whose count changed) and dense destinations (the RCS grew) move.
    int32_t f0 = 0;
    int64_t t_keep = 0;   // the seed's targets kept
    if (seed && seed->row_tgt.size() == (size_t)seed->nFB + 1 && seed->dense == pl.dense && seed->D == D &&
        seed->gram_seg == pl.gram_seg && seed->iw == pl.iw && seed->nintr == nintr && world == 1) {
        int32_t f = std::min(seed->ncam, ncam);
        for (int32_t c = 0; c < ngrp; ++c)
            if (pl.group_off[c] >= pl.reused_chunks) f = std::min(f, g_lo[c]);
        for (int64_t g = pl.reused_gpts; g < pl.n_gpt; ++g) f = std::min(f, p_lo[g]);
        if (f > 0 && f <= seed->nFB) {
            t_keep = seed->row_tgt[f];
            const bool tail = t_keep < (int64_t)seed->targets.size();
            if (tail && seed->targets[t_keep].c_begin == BS(kMc, f) && seed->targets[t_keep].p_begin == BS(kMp, f) &&
                (int64_t)seed->terms.size() >= BS(kMc, f) && (int64_t)seed->pterms.size() >= BS(kMp, f))
                f0 = f;
        }
    }
    if (f0 > 0) {
        BAHostPlan& q = *seed;
        pl.terms = std::move(q.terms);
        pl.pterms = std::move(q.pterms);
        pl.targets = std::move(q.targets);
        pl.targets.resize(t_keep);
        const int64_t q_u = std::max<int64_t>(q.n_group(), 1) * kTileR * kTileR,
                      q_ub = q_u + fw * fw * q.n_img * kGramSeg, q_ucn = q_ub + fw * q.n_img * kGramSeg;
        const int64_t du = o_u - q_u, dub = o_ub - q_ub, ducn = o_ucn - q_ucn;
        FlatTerm* T = pl.terms.data();
        parallel_ranges(BS(kMc, f0), [&](int64_t a0, int64_t a1, int) {
            for (int64_t k = a0; k < a1; ++k) {
                const int64_t o = T[k].off;
                T[k].off = o + (o >= q_ucn ? ducn : o >= q_ub ? dub : o >= q_u ? du : 0);
            }
        });
        if (!band)
            for (ReduceTarget& t : pl.targets) {   // camera rows: (fa, fb) columns unchanged, the row stride grew
                const int64_t ca = t.dst / q.nF, cb = t.dst % q.nF;
                t.dst = ca * pl.nF + cb;
                t.ld = (int32_t)pl.nF;
            }
    } else {
        pl.targets.clear();
    }
    grow_to(pl.terms, n_terms);
    grow_to(pl.pterms, n_pterms);
    tm.mark("terms_count");

    // ---- targets and terms, by row ranges ----------------------------------
    // matrix targets of row fa: band -- the band blocks (fa, fa-d), d from
    // min(D, fa) down to 0; an intrinsics row ncam+m: the arrow (m, i) for
    // every camera, then per corner column l <= m the transposed (l, m) (l <
    // m) and (m, l) -- the order a stable sort of the targets by key gives.
    // Dense: every block (fa, fb <= fa) that receives a term.
    auto row_slots = [&](int32_t f) -> int64_t {
        if (!band) return (int64_t)f + 1;
        return f < ncam ? std::min(D, f) + 1 : ncam + 2 * (f - ncam) + 1;
    };
    // slot of (fa, fb) within row fa; *second: a transposed twin at slot - 1
    auto slot_of = [&](int32_t fa, int32_t fb) -> int64_t {
        if (!band) return fb;
        if (fa < ncam) return fb - (fa - std::min(D, fa));
        if (fb < ncam) return fb;
        return ncam + 2 * (fb - ncam) + (fb != fa ? 1 : 0);   // the (fa, fb) target; its twin precedes it
    };
    auto make_target = [&](int32_t fa, int64_t s) {
        ReduceTarget t{};
        if (!band) {
            const int32_t fb = (int32_t)s;
            t.dst = col_of_fb(fa) * pl.nF + col_of_fb(fb);
            t.dst_kind = kDstDense;
            t.rows = size_of_fb(fa); t.cols = size_of_fb(fb); t.ld = (int32_t)pl.nF;
        } else if (fa < ncam) {
            const int d = std::min(D, fa) - (int)s;
            t.dst = ((int64_t)fa * Dp + d) * 36;
            t.dst_kind = kDstBand;
            t.rows = 6; t.cols = 6; t.ld = 6;
        } else if (s < ncam) {
            t.dst = ((int64_t)(fa - ncam) * ncam + s) * 6 * pl.iw;
            t.dst_kind = kDstArrow;
            t.rows = pl.iw; t.cols = 6; t.ld = 6;
        } else {
            const int m = fa - ncam, u = (int)(s - ncam), lp = u / 2;
            const bool trans = (u & 1) == 0 && lp < m;
            const int k = trans ? lp : m, l = trans ? m : lp;
            t.dst = ((int64_t)k * nintr + l) * pl.iw * pl.iw;
            t.dst_kind = kDstCorner;
            t.rows = pl.iw; t.cols = pl.iw; t.ld = pl.iw;
        }
        return t;
    };
    // row ranges of about equal work (terms, plus the row's targets)
    // (matrix rows f0.. here; every row's vector terms below)
    auto row_cuts = [&](int32_t fa0, bool matrix) {
        std::vector<int32_t> cut{fa0};
        int64_t tot = 0;
        std::vector<int64_t> w(nFB);
        for (int32_t f = fa0; f < nFB; ++f) {
            w[f] = matrix ? RC(kMc, f) + RC(kMp, f) + row_slots(f) : RC(kVc, f) + RC(kVp, f) + 2 * RC(kVb, f);
            tot += w[f];
        }
        const int nt = tot < 65536 ? 1 : std::min<int>(PlanPool::width(), std::max(1, nFB - fa0));
        int64_t acc = 0;
        for (int32_t f = fa0; f < nFB; ++f) {
            acc += w[f];
            if ((int)cut.size() < nt && acc * nt >= (int64_t)cut.size() * tot && f + 1 < nFB) cut.push_back(f + 1);
        }
        cut.push_back(nFB);
        return cut;
    };
    const std::vector<int32_t> cut = row_cuts(f0, true);
    const int nseg = (int)cut.size() - 1;
    std::vector<std::vector<ReduceTarget>> seg_targets(nseg);
    std::vector<std::vector<int32_t>> seg_rows(nseg);   // each row's first target within its segment
    std::vector<int> seg_rc(nseg, SFM_OK);
    parallel_segments(nseg, [&](int sg) {
        seg_rc[sg] = guarded([&] {
            const int32_t r0 = cut[sg], r1 = cut[sg + 1];
            std::vector<int64_t> sbase(r1 - r0 + 1, 0);   // first slot of each row
            for (int32_t f = r0; f < r1; ++f) sbase[f - r0 + 1] = sbase[f - r0] + row_slots(f);
            const int64_t ns = sbase[r1 - r0];
            // per slot: sum / product term counts, then write cursors
            std::vector<int64_t> cs(ns, 0), ps(ns, 0);
            auto S = [&](int32_t fa, int32_t fb) { return sbase[fa - r0] + slot_of(fa, fb); };
            auto in = [&](int32_t f) { return f >= r0 && f < r1; };
            // (1) counts
            for (const ImgSrc& s : isrc) {
                if (s.cb >= 0 && in(s.cb)) cs[S(s.cb, s.cb)] += gseg;
                if (s.fq >= 0 && in(s.fq)) {
                    if (s.cb >= 0) cs[S(s.fq, s.cb)] += gseg;
                    cs[S(s.fq, s.fq)] += gseg;
                }
            }
            for (int32_t c = 0; c < ngrp; ++c) {
                if (g_hi[c] < r0 || g_lo[c] >= r1) continue;
                const ChunkDesc& cd = grp(c);
                for (int a = 0; a < cd.n_slots; ++a) {
                    const int32_t fa = gfb[(size_t)c * kMaxSlots + a];
                    if (!in(fa)) continue;
                    for (int b = 0; b < cd.n_slots; ++b) {
                        const int32_t fb = gfb[(size_t)c * kMaxSlots + b];
                        if (fa < fb || !held(fa, fb)) continue;
                        const int64_t q = S(fa, fb);
                        cs[q]++;
                        if (twice(fa, fb)) cs[q - 1]++;
                    }
                }
            }
            for (int64_t g = 0; g < pl.n_gpt; ++g) {
                if (p_hi[g] < r0 || p_lo[g] >= r1) continue;
                const int32_t k0 = pl.gblk_off[g], k1 = pl.gblk_off[g + 1];
                for (int32_t a = k0; a < k1; ++a) {
                    const int32_t fa = pfb[a];
                    if (fa < r0) continue;
                    if (fa >= r1) break;
                    for (int32_t b = k0; b <= a; ++b) {
                        const int32_t fb = pfb[b];
                        const int64_t q = S(fa, fb);
                        ps[q]++;
                        if (twice(fa, fb)) ps[q - 1]++;
                    }
                }
            }
            // (2) targets in slot order; the counts become write cursors
            auto& tg = seg_targets[sg];
            seg_rows[sg].resize(r1 - r0);
            int64_t c_at = BS(kMc, r0), p_at = BS(kMp, r0);
            for (int32_t f = r0; f < r1; ++f)
                for (int64_t s = (seg_rows[sg][f - r0] = (int32_t)tg.size(), 0); s < row_slots(f); ++s) {
                    const int64_t q = sbase[f - r0] + s;
                    const int64_t nc = cs[q], np = ps[q];
                    cs[q] = c_at;
                    ps[q] = p_at;
                    if (!band && nc == 0 && np == 0) continue;
                    ReduceTarget t = make_target(f, s);
                    t.c_begin = (int32_t)c_at; t.c_end = (int32_t)(c_at + nc);
                    t.p_begin = (int32_t)p_at; t.p_end = (int32_t)(p_at + np);
                    c_at += nc;
                    p_at += np;
                    tg.push_back(t);
                }
            // (3) the terms, sources in order
            FlatTerm* T = pl.terms.data();
            PTerm* PT = pl.pterms.data();
            auto put = [&](int64_t q, bool tw, ReduceTerm r) {
                T[cs[q]++] = flat(r, false);
                if (tw) {
                    std::swap(r.roff, r.coff);
                    T[cs[q - 1]++] = flat(r, false);
                }
            };
            auto put_p = [&](int64_t q, bool tw, PTerm r) {
                PT[ps[q]++] = r;
                if (tw) {
                    std::swap(r.za, r.zb);
                    PT[ps[q - 1]++] = r;
                }
            };
            for (const ImgSrc& s : isrc)
                for (int g = 0; g < gseg; ++g) {
                    const int32_t idx = s.img * gseg + g;
                    if (s.cb >= 0 && in(s.cb)) put(S(s.cb, s.cb), false, ReduceTerm{kSrcU, idx, 0, 0, 1.f});
                    if (s.fq >= 0 && in(s.fq)) {
                        if (s.cb >= 0) put(S(s.fq, s.cb), false, ReduceTerm{kSrcU, idx, 6, 0, 1.f});
                        put(S(s.fq, s.fq), false, ReduceTerm{kSrcU, idx, 6, 6, 1.f});
                    }
                }
            for (int32_t c = 0; c < ngrp; ++c) {
                if (g_hi[c] < r0 || g_lo[c] >= r1) continue;
                const ChunkDesc& cd = grp(c);
                for (int a = 0; a < cd.n_slots; ++a) {
                    const int32_t fa = gfb[(size_t)c * kMaxSlots + a];
                    if (!in(fa)) continue;
                    for (int b = 0; b < cd.n_slots; ++b) {
                        const int32_t fb = gfb[(size_t)c * kMaxSlots + b];
                        if (fa < fb || !held(fa, fb)) continue;
                        put(S(fa, fb), twice(fa, fb),
                            ReduceTerm{kSrcTile, c, (int16_t)cd.slot_row[a], (int16_t)cd.slot_row[b], 1.f});
                    }
                }
            }
            for (int64_t g = 0; g < pl.n_gpt; ++g) {
                if (p_hi[g] < r0 || p_lo[g] >= r1) continue;
                const int32_t k0 = pl.gblk_off[g], k1 = pl.gblk_off[g + 1];
                const int64_t zb = pl.gz_off[g];
                for (int32_t a = k0; a < k1; ++a) {
                    const int32_t fa = pfb[a];
                    if (fa < r0) continue;
                    if (fa >= r1) break;
                    for (int32_t b = k0; b <= a; ++b) {
                        const int32_t fb = pfb[b];
                        put_p(S(fa, fb), twice(fa, fb), PTerm{(int32_t)(zb + pl.gblk_z[a]), (int32_t)(zb + pl.gblk_z[b])});
                    }
                }
            }
            return SFM_OK;
        });
    });
    for (int sg = 0; sg < nseg; ++sg)
        if (seg_rc[sg] != SFM_OK) throw SfmError{seg_rc[sg]};
    tm.mark("terms");
    // ---- every row's vector terms (rhs sum / product, bF, cnF): the image
    // slices, then tile row 79 (-Z w) in group order, then the general points'
    // w, per row -- the order of its matrix terms' sources -----------------------
    {
        const std::vector<int32_t> vcut = row_cuts(0, false);
        const int nv = (int)vcut.size() - 1;
        std::vector<int> v_rc(nv, SFM_OK);
        parallel_segments(nv, [&](int sg) {
            v_rc[sg] = guarded([&] {
                const int32_t r0 = vcut[sg], r1 = vcut[sg + 1];
                auto in = [&](int32_t f) { return f >= r0 && f < r1; };
                FlatTerm* T = pl.terms.data();
                PTerm* PT = pl.pterms.data();
                std::vector<int64_t> vcur(4 * (size_t)(r1 - r0));
                for (int32_t f = r0; f < r1; ++f) {
                    vcur[4 * (f - r0) + 0] = n_mc + BS(kVc, f);
                    vcur[4 * (f - r0) + 1] = n_mp + BS(kVp, f);
                    vcur[4 * (f - r0) + 2] = n_mc + n_vc + BS(kVb, f);
                    vcur[4 * (f - r0) + 3] = n_mc + n_vc + n_vb + BS(kVb, f);
                }
                auto put_v = [&](int32_t f, int16_t ro, int32_t idx) {
                    int64_t* v = &vcur[4 * (f - r0)];
                    T[v[0]++] = flat(ReduceTerm{kSrcUb, idx, ro, 0, 1.f}, true);
                    T[v[2]++] = flat(ReduceTerm{kSrcUb, idx, ro, 0, 1.f}, true);
                    T[v[3]++] = flat(ReduceTerm{kSrcUcn, idx, ro, 0, 1.f}, true);
                };
                for (const ImgSrc& s : isrc)
                    for (int g = 0; g < gseg; ++g) {
                        const int32_t idx = s.img * gseg + g;
                        if (s.cb >= 0 && in(s.cb)) put_v(s.cb, 0, idx);
                        if (s.fq >= 0 && in(s.fq)) put_v(s.fq, 6, idx);
                    }
                for (int32_t c = 0; c < ngrp; ++c) {
                    if (g_hi[c] < r0 || g_lo[c] >= r1) continue;
                    const ChunkDesc& cd = grp(c);
                    for (int a = 0; a < cd.n_slots; ++a) {
                        const int32_t fa = gfb[(size_t)c * kMaxSlots + a];
                        if (in(fa))   // rhs contribution (-Z w) from tile row 79
                            T[vcur[4 * (fa - r0)]++] =
                                flat(ReduceTerm{kSrcTile, c, (int16_t)kTileWRow, (int16_t)cd.slot_row[a], 1.f}, true);
                    }
                }
                for (int64_t g = 0; g < pl.n_gpt; ++g) {
                    if (p_hi[g] < r0 || p_lo[g] >= r1) continue;
                    const int32_t k0 = pl.gblk_off[g], k1 = pl.gblk_off[g + 1];
                    const int64_t zb = pl.gz_off[g], wz = pl.gz_off[g + 1] - 3;
                    for (int32_t a = k0; a < k1; ++a) {
                        const int32_t fa = pfb[a];
                        if (fa < r0) continue;
                        if (fa >= r1) break;
                        PT[vcur[4 * (fa - r0) + 1]++] = PTerm{(int32_t)(zb + pl.gblk_z[a]), (int32_t)wz};
                    }
                }
                return SFM_OK;
            });
        });
        for (int sg = 0; sg < nv; ++sg)
            if (v_rc[sg] != SFM_OK) throw SfmError{v_rc[sg]};
    }
    tm.mark("vector_terms");
    {
        // the matrix targets: the seed's rows before f0 (pl.targets already),
        // then this plan's; every row's first target for the next grown plan
        size_t nt = pl.targets.size() + 3 * (size_t)nFB;
        for (const auto& v : seg_targets) nt += v.size();
        pl.targets.reserve(nt);
        for (const auto& v : seg_targets) pl.targets.insert(pl.targets.end(), v.begin(), v.end());
        pl.row_tgt.assign(nFB + 1, 0);
        if (f0 > 0) std::copy(seed->row_tgt.begin(), seed->row_tgt.begin() + f0, pl.row_tgt.begin());
        int64_t at = t_keep;
        for (int sg = 0; sg < nseg; ++sg) {
            for (int32_t f = cut[sg]; f < cut[sg + 1]; ++f) pl.row_tgt[f] = (int32_t)(at + seg_rows[sg][f - cut[sg]]);
            at += (int64_t)seg_targets[sg].size();
        }
        pl.row_tgt[nFB] = (int32_t)at;
    }
    // vectors: rhs = bF - Z w, bF, cnF, per F block in order
    for (int pass = 0; pass < 3; ++pass)
        for (int32_t fb = 0; fb < nFB; ++fb) {
            ReduceTarget t{};
            t.dst = col_of_fb(fb);
            t.dst_kind = pass == 0 ? kDstRhs : pass == 1 ? kDstBF : kDstCnF;
            t.rows = size_of_fb(fb); t.cols = 1; t.ld = 1;
            const int64_t c0 = pass == 0 ? n_mc + BS(kVc, fb) : n_mc + n_vc + (pass - 1) * n_vb + BS(kVb, fb);
            const int64_t nc = pass == 0 ? RC(kVc, fb) : RC(kVb, fb);
            t.c_begin = (int32_t)c0; t.c_end = (int32_t)(c0 + nc);
            if (pass == 0) {
                t.p_begin = (int32_t)(n_mp + BS(kVp, fb));
                t.p_end = (int32_t)(t.p_begin + RC(kVp, fb));
            } else {
                t.p_begin = t.p_end = (int32_t)n_pterms;
            }
            pl.targets.push_back(t);
        }
    pl.zero_targets.clear();
    if (world > 1) {
        // a shard gathers terms only into the blocks its points touch (about
        // 1/world of the band); the others, which other shards write, go to a
        // zero list that the reduce launch clears beside the real targets.
        // (Dense plans list only this shard's blocks, so the solver clears
        // their whole system before each reduce instead.)
        size_t w = 0;
        for (size_t t = 0; t < pl.targets.size(); ++t) {
            const ReduceTarget& T = pl.targets[t];
            if (T.c_begin != T.c_end || T.p_begin != T.p_end) pl.targets[w++] = T;
            else pl.zero_targets.push_back(T);
        }
        pl.targets.resize(w);
    }
    tm.mark("targets");
}

}  // namespace

}  // namespace sfm

namespace sfm {

uint64_t plan_digest(const BAHostPlan& h, bool with_uv) {
    uint64_t x = 1469598103934665603ull;
    auto bytes = [&](const void* p, size_t n) {
        const auto* b = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; ++i) x = (x ^ b[i]) * 1099511628211ull;
    };
    static const bool parts = std::getenv("SFM_PLAN_DIGEST_PARTS") != nullptr;   // (diagnostic: per array)
    int part = 0;
    auto vec = [&](const auto& v) {   // (element types without padding)
        const uint64_t n = v.size();
        const uint64_t x0 = x;
        x = 1469598103934665603ull;
        bytes(&n, sizeof n);
        if (n) bytes(v.data(), n * sizeof(v[0]));
        if (parts) std::fprintf(stderr, "[digest] part %d n %llu -> %016llx\n", part, (unsigned long long)n,
                                (unsigned long long)x);
        const uint64_t xp = x;
        x = x0;
        bytes(&xp, sizeof xp);
        ++part;
    };
    vec(h.targets); vec(h.zero_targets); vec(h.terms); vec(h.pterms); vec(h.chunks); vec(h.group_off);
    vec(h.pt_off); vec(h.obs_img); vec(h.obs_slot); vec(h.gobs_perm);
    vec(h.gblk_off); vec(h.gblk_col); vec(h.gblk_z); vec(h.gz_off); vec(h.zbatch); vec(h.zlong);
    vec(h.spt_global); vec(h.img_obs_ptr); vec(h.gram_img);
    vec(h.cam_blk); vec(h.intr_blk); vec(h.blk_img); vec(h.blk_intr); vec(h.img_colc); vec(h.img_coli);
    if (with_uv) vec(h.obs_uv);
    const int64_t sc[] = {h.n_img, h.n_intr, h.n_pt, h.n_obs, h.ncam, h.nintr, h.D, h.nb, h.na, h.nF, h.iw,
                          h.nFB, h.dense, h.n_sdense, h.n_spt, h.n_sobs, h.n_cpt, h.n_gpt, h.gram_seg, h.n_z,
                          h.gz_max, h.tile_nt, h.n_sband, h.n_sarrow, h.n_scorner, h.schur_flops, h.schur_bytes};
    bytes(sc, sizeof sc);
    return x;
}

}  // namespace sfm

extern "C" int sfm_ba_grown_digest(const sfm_ba_problem* prev, const sfm_ba_problem* prob, uint64_t* digest_fresh,
                                   uint64_t* digest_grown, int64_t* reused) {
    using namespace sfm;
    return guarded([&] {
        SFM_REQUIRE(prev && prob && digest_fresh && digest_grown && reused, SFM_ERR_INVALID_ARG, "bad arguments");
        BAHostPlan seed, grown, fresh;
        build_plan(*prev, 0, 1, seed);
        GrowPrev gp;
        gp.n_img = prev->n_img; gp.n_intr = prev->n_intr; gp.const_img = prev->const_img; gp.model = prev->camera_model;
        gp.n_pt = prev->n_pt; gp.n_obs = prev->n_obs;
        gp.pt_offsets = prev->pt_offsets; gp.obs_img = prev->obs_img; gp.img_intr = prev->img_intr;
        const bool ok = build_plan_grown(*prob, gp, seed, grown);
        build_plan(*prob, 0, 1, fresh);
        *digest_fresh = plan_digest(fresh, false);
        *digest_grown = ok ? plan_digest(grown, false) : 0;
        *reused = ok ? grown.reused_pts : -1;
        return SFM_OK;
    });
}

extern "C" int sfm_ba_intr_width(int32_t camera_model) {
    switch (camera_model) {
        case SFM_CAM_PINHOLE: case SFM_CAM_SNAVELY: return 4;
        case SFM_CAM_RADIAL3: return 6;
        default: return 0;
    }
}

extern "C" int sfm_ba_partition(const sfm_ba_problem* prob, int32_t world_size, int64_t* order,
                                int64_t* bounds) {
    using namespace sfm;
    return guarded([&] {
        SFM_REQUIRE(prob && order && bounds && world_size >= 1, SFM_ERR_INVALID_ARG, "bad arguments");
        const std::vector<int32_t> cam_blk = camera_blocks(*prob, nullptr, nullptr);
        std::vector<int64_t> ord, bnd;
        partition_points(*prob, cam_blk, world_size, ord, bnd);
        std::copy(ord.begin(), ord.end(), order);
        std::copy(bnd.begin(), bnd.end(), bounds);
        return SFM_OK;
    });
}

extern "C" int sfm_ba_describe(const sfm_ba_problem* prob, int32_t rank, int32_t world_size,
                               sfm_ba_plan_shape* out) {
    using namespace sfm;
    return guarded([&] {
        SFM_REQUIRE(prob && out && world_size >= 1 && rank >= 0 && rank < world_size, SFM_ERR_INVALID_ARG,
                    "bad arguments");
        BAHostPlan h;
        build_plan(*prob, rank, world_size, h);
        if (std::getenv("SFM_PLAN_DIGEST")) {
            // diagnostic: FNV-1a of every plan array (planner refactors must
            // keep it; the arrays' element types carry no padding)
            auto fnv = [](const auto& v) {
                uint64_t x = 1469598103934665603ull;
                const auto* b = reinterpret_cast<const unsigned char*>(v.data());
                for (size_t i = 0; i < v.size() * sizeof(v[0]); ++i) x = (x ^ b[i]) * 1099511628211ull;
                return (unsigned long long)x;
            };
            std::fprintf(stderr,
                         "[digest] targets %016llx terms %016llx pterms %016llx chunks %016llx obs %016llx %016llx "
                         "%016llx gen %016llx %016llx %016llx %016llx %016llx %016llx order %016llx %016llx\n",
                         fnv(h.targets), fnv(h.terms), fnv(h.pterms), fnv(h.chunks), fnv(h.obs_img), fnv(h.obs_slot),
                         fnv(h.obs_uv), fnv(h.gblk_off), fnv(h.gblk_col), fnv(h.gblk_z), fnv(h.gz_off), fnv(h.zbatch),
                         fnv(h.zlong), fnv(h.spt_global), fnv(h.img_obs_ptr));
        }
        *out = sfm_ba_plan_shape{};
        out->n_chunks = (int32_t)h.chunks.size();
        out->band_blocks = h.D;
        out->dense = h.dense ? 1 : 0;
        out->n_cam_active = h.ncam;
        out->n_intr_active = h.nintr;
        out->tile_rows = 16 * h.tile_nt;
        out->n_chunk_pts = h.n_cpt;
        out->n_general_pts = h.n_gpt;
        out->rcs_dim = h.nF;
        out->n_targets = (int64_t)h.targets.size();
        out->n_terms = (int64_t)h.terms.size();
        out->n_pterms = (int64_t)h.pterms.size();
        return SFM_OK;
    });
}
