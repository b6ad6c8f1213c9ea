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
#include <cstdlib>
#include <climits>
#include <map>
#include <numeric>
#include <thread>

#include "common.h"

namespace sfm {

namespace {

// Split [0, n) into contiguous ranges over up to 16 host threads (results are
// independent of the split: every range writes its own outputs).
template <class F>
void parallel_ranges(int64_t n, F&& fn) {
    const int64_t hw = std::max<int64_t>(1, std::min<int64_t>(16, std::thread::hardware_concurrency()));
    const int64_t nt = n < 65536 ? 1 : hw;
    if (nt <= 1) {
        fn(0, n, 0);
        return;
    }
    std::vector<std::thread> th;
    for (int64_t t = 1; t < nt; ++t) th.emplace_back([&, t] { fn(n * t / nt, n * (t + 1) / nt, (int)t); });
    fn(0, n / nt, 0);
    for (auto& x : th) x.join();
}

void active_sets(const sfm_ba_problem& P, BAHostPlan& pl) {
    pl.cam_blk.assign(P.n_img, -1);
    pl.intr_blk.assign(P.n_intr, -1);
    std::vector<char> cu(P.n_img, 0), iu(P.n_intr, 0);
    for (int64_t o = 0; o < P.n_obs; ++o) {
        cu[P.obs_img[o]] = 1;
        iu[P.img_intr[P.obs_img[o]]] = 1;
    }
    for (int i = 0; i < P.n_img; ++i)
        if (cu[i] && i != P.const_img) { pl.cam_blk[i] = pl.ncam++; pl.blk_img.push_back(i); }
    for (int q = 0; q < P.n_intr; ++q)
        if (iu[q]) { pl.intr_blk[q] = pl.nintr++; pl.blk_intr.push_back(q); }
    pl.nb = 6LL * pl.ncam;
    pl.na = 4LL * pl.nintr;
    pl.nF = pl.nb + pl.na;
    pl.img_colc.assign(P.n_img, -1);
    pl.img_coli.assign(P.n_img, -1);
    pl.img_intr.assign(P.img_intr, P.img_intr + P.n_img);
    for (int i = 0; i < P.n_img; ++i) {
        if (pl.cam_blk[i] >= 0) pl.img_colc[i] = 6 * pl.cam_blk[i];
        const int q = pl.intr_blk[P.img_intr[i]];
        if (q >= 0) pl.img_coli[i] = (int32_t)(pl.nb + 4 * q);
    }
}

}  // namespace

void partition_points(const sfm_ba_problem& P, const std::vector<int32_t>& cam_blk, int world,
                      std::vector<int64_t>& order, std::vector<int64_t>& bounds) {
    struct Key { int32_t lo, hi; int64_t id; };
    std::vector<Key> keys(P.n_pt);
    for (int64_t p = 0; p < P.n_pt; ++p) {
        int lo = INT_MAX, hi = -1;
        for (int64_t o = P.pt_offsets[p]; o < P.pt_offsets[p + 1]; ++o) {
            const int b = cam_blk[P.obs_img[o]];
            if (b >= 0) { lo = std::min(lo, b); hi = std::max(hi, b); }
        }
        keys[p] = {lo, hi, p};
    }
    std::stable_sort(keys.begin(), keys.end(), [](const Key& a, const Key& b) {
        return a.lo != b.lo ? a.lo < b.lo : a.hi < b.hi;
    });
    order.resize(P.n_pt);
    for (int64_t k = 0; k < P.n_pt; ++k) order[k] = keys[k].id;
    bounds.assign(world + 1, P.n_pt);
    bounds[0] = 0;
    int64_t acc = 0, r = 1;
    for (int64_t k = 0; k < P.n_pt && r < world; ++k) {
        const int64_t p = order[k];
        acc += P.pt_offsets[p + 1] - P.pt_offsets[p];
        while (r < world && acc * world >= r * P.n_obs) bounds[r++] = k + 1;
    }
}

void build_plan(const sfm_ba_problem& P, int rank, int world, BAHostPlan& pl) {
    SFM_REQUIRE(P.n_img >= 1 && P.n_intr >= 1 && P.n_pt >= 0 && P.n_obs >= 0 &&
                    P.pt_offsets && (P.n_obs == 0 || (P.obs_img && P.obs_uv)) && P.img_intr,
                SFM_ERR_INVALID_ARG, "incomplete BA problem");
    SFM_REQUIRE(P.pt_offsets[0] == 0 && P.pt_offsets[P.n_pt] == P.n_obs, SFM_ERR_INVALID_ARG,
                "pt_offsets must run from 0 to n_obs");
    SFM_REQUIRE(P.n_obs < INT32_MAX && P.n_pt < INT32_MAX, SFM_ERR_UNSUPPORTED,
                "more than 2^31 observations per process");
    for (int64_t p = 0; p < P.n_pt; ++p)
        SFM_REQUIRE(P.pt_offsets[p + 1] >= P.pt_offsets[p], SFM_ERR_INVALID_ARG,
                    "pt_offsets not monotone at point %lld", (long long)p);
    for (int64_t o = 0; o < P.n_obs; ++o)
        SFM_REQUIRE(P.obs_img[o] >= 0 && P.obs_img[o] < P.n_img, SFM_ERR_INVALID_ARG,
                    "obs %lld references image %d", (long long)o, P.obs_img[o]);
    for (int i = 0; i < P.n_img; ++i)
        SFM_REQUIRE(P.img_intr[i] >= 0 && P.img_intr[i] < P.n_intr, SFM_ERR_INVALID_ARG,
                    "image %d references intrinsics %d", i, P.img_intr[i]);
    SFM_REQUIRE(P.const_img >= -1 && P.const_img < P.n_img, SFM_ERR_INVALID_ARG, "bad const_img");
    SFM_REQUIRE(P.camera_model == SFM_CAM_PINHOLE || P.camera_model == SFM_CAM_SNAVELY, SFM_ERR_INVALID_ARG,
                "unknown camera_model %d", P.camera_model);

    pl.n_img = P.n_img; pl.n_intr = P.n_intr; pl.n_pt = P.n_pt; pl.n_obs = P.n_obs;
    pl.rank = rank; pl.world = world;
    active_sets(P, pl);
    SFM_REQUIRE(pl.nintr <= 4, SFM_ERR_UNSUPPORTED,
                "%d active intrinsic blocks; this build supports up to 4 (dense arrow)", pl.nintr);

    // band half-width (blocks) over active cameras; duplicate views rejected
    int32_t D = 0;
    for (int64_t p = 0; p < P.n_pt; ++p) {
        int lo = INT_MAX, hi = -1;
        for (int64_t o = P.pt_offsets[p]; o < P.pt_offsets[p + 1]; ++o) {
            for (int64_t o2 = P.pt_offsets[p]; o2 < o; ++o2)
                SFM_REQUIRE(P.obs_img[o2] != P.obs_img[o], SFM_ERR_UNSUPPORTED,
                            "point %lld observed twice by image %d", (long long)p, P.obs_img[o]);
            const int b = pl.cam_blk[P.obs_img[o]];
            if (b >= 0) { lo = std::min(lo, b); hi = std::max(hi, b); }
        }
        if (hi >= 0) D = std::max(D, hi - lo);
    }
    pl.D = D;

    partition_points(P, pl.cam_blk, world, pl.order, pl.bounds);

    // ---- shard arrays ------------------------------------------------------
    const int64_t b0 = pl.bounds[rank], b1 = pl.bounds[rank + 1];
    pl.n_spt = b1 - b0;
    pl.spt_global.assign(pl.order.begin() + b0, pl.order.begin() + b1);
    pl.pt_off.assign(pl.n_spt + 1, 0);
    for (int64_t k = 0; k < pl.n_spt; ++k) {
        const int64_t p = pl.spt_global[k];
        pl.pt_off[k + 1] = pl.pt_off[k] + (int32_t)(P.pt_offsets[p + 1] - P.pt_offsets[p]);
    }
    pl.n_sobs = pl.pt_off[pl.n_spt];
    pl.obs_img.resize(pl.n_sobs);
    pl.obs_pt.resize(pl.n_sobs);
    pl.obs_uv.resize(2 * pl.n_sobs);
    pl.obs_slot.assign(pl.n_sobs, 0);
    parallel_ranges(pl.n_spt, [&](int64_t k0, int64_t k1, int) {
        for (int64_t k = k0; k < k1; ++k) {
            const int64_t p = pl.spt_global[k];
            for (int64_t o = P.pt_offsets[p], s = pl.pt_off[k]; o < P.pt_offsets[p + 1]; ++o, ++s) {
                pl.obs_img[s] = P.obs_img[o];
                pl.obs_pt[s] = (int32_t)k;
                pl.obs_uv[2 * s] = P.obs_uv[2 * o];
                pl.obs_uv[2 * s + 1] = P.obs_uv[2 * o + 1];
            }
        }
    });

    // ---- Schur chunks --------------------------------------------------------
    // Greedy over shard points: a chunk's F blocks (camera 6 rows, intrinsics 4
    // rows) must fit `cap` rows of its tile: 64 (4x4 MFMA tiles, -Zw on the
    // VALU) or 76 (5x5 tiles, -Zw in row 79).  The 64-row form does 2/3 of the
    // MFMA work per point; it is used unless it would need many more chunks.
    // 128 points per chunk: ~2x the co-resident waves of the chip at C4 size,
    // so the last round of chunks is short (256 measured 17% slower).
    // A shard too small to give every wave slot of the chip a 128-point chunk
    // (a landmark shard at N = 4, 8) gets shorter chunks instead, down to 16
    // points: the Schur pass takes about one chunk's latency once the chunks
    // fit in one round, so 2048 chunks (8 waves per CU) keep it dividing by N.
    constexpr int64_t kTargetChunks = 2048;
    int chunk_pts = (int)std::max<int64_t>(16, std::min<int64_t>(kChunkPts, (pl.n_spt + kTargetChunks - 1) / kTargetChunks));
    if (const char* e = std::getenv("SFM_BA_CHUNK_PTS")) chunk_pts = std::max(1, std::min(kChunkPts, std::atoi(e)));   // tuning override
    auto make_chunks = [&](int cap, std::vector<ChunkDesc>& chunks_out, std::vector<int32_t>& slot_out) -> int64_t {
        int64_t flops = 0;
        slot_out.assign(pl.n_sobs, 0);
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
        auto close = [&](int32_t p_end) {
            cd.pt_end = p_end;
            cd.obs_end = pl.pt_off[p_end];
            cd.n_slots = (int32_t)(cams.size() + intrs.size());
            cd.n_cams = (int32_t)dcams.size();
            cd.n_intr = (int32_t)intrs.size();
            chunks_out.push_back(cd);
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
        if (pl.n_spt > 0) reset(0);
        for (int32_t k = 0; k < (int32_t)pl.n_spt; ++k) {
            const int32_t nobs = pl.pt_off[k + 1] - pl.pt_off[k];
            SFM_REQUIRE(nobs <= kSubObs, SFM_ERR_UNSUPPORTED, "point with %d observations (> %d)",
                        nobs, kSubObs);
            Small pc, pi, pd;
            for (int32_t s = pl.pt_off[k]; s < pl.pt_off[k + 1]; ++s) {
                const int img = pl.obs_img[s];
                if (pl.cam_blk[img] >= 0) pc.push_back(img);
                pd.push_back(img);
                const int q = P.img_intr[img];
                if (!pi.has(q)) pi.push_back(q);
            }
            const int own = 6 * (int)pc.size() + 4 * (int)pi.size();
            SFM_REQUIRE(own <= cap && (int)pd.size() <= kCamSlots && (int)pi.size() <= kIntrSlots,
                        SFM_ERR_UNSUPPORTED,
                        "point %lld spans %d F rows / %d images (> %d / %d): track too long for this build",
                        (long long)pl.spt_global[k], own, (int)pd.size(), cap, kCamSlots);
            int add = 0, add_slots = 0, add_d = 0, add_i = 0;
            for (int img : pc) if (cam_slot[img] < 0) { add += 6; ++add_slots; }
            for (int q : pi) if (intr_idx[q] < 0) { add += 4; ++add_slots; ++add_i; }
            for (int img : pd) if (dcam_idx[img] < 0) ++add_d;
            const bool full = k > cd.pt_begin &&
                              (rows + add > cap || k - cd.pt_begin >= chunk_pts ||
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
                    cd.slot_col[s] = (int32_t)(pl.nb + 4 * pl.intr_blk[q]);
                    cd.intr_id[t] = q; cd.intr_row[t] = rows; cd.intr_col[t] = cd.slot_col[s];
                    rows += 4;
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
            // algorithmic flops: the symmetric Z Z' over the
            // point's own F rows (r(r+1)/2 entries x 3 x 2 = 3 r (r+1)), the
            // linearisation (600 per observation) and the point block (V, its
            // factor, M = Jx L^-T, Z = J' M: 180 per observation + 30)
            const int64_t nfp = own;
            flops += 3LL * nfp * (nfp + 1) + 780LL * nobs + 30;
        }
        if (pl.n_spt > 0) close((int32_t)pl.n_spt);
        return flops;
    };
    int max_own = 0, max_obs = 0;
    for (int64_t k = 0; k < pl.n_spt; ++k) {
        max_obs = std::max(max_obs, pl.pt_off[k + 1] - pl.pt_off[k]);
        int nc = 0;
        std::vector<int> pi;
        for (int32_t s = pl.pt_off[k]; s < pl.pt_off[k + 1]; ++s) {
            if (pl.cam_blk[pl.obs_img[s]] >= 0) ++nc;
            const int q = P.img_intr[pl.obs_img[s]];
            if (std::find(pi.begin(), pi.end(), q) == pi.end()) pi.push_back(q);
        }
        max_own = std::max(max_own, 6 * nc + 4 * (int)pi.size());
    }
    int64_t flops = 0;
    pl.tile_nt = 5;
    // the 64-row kernel walks 48-observation batches (ba_kernels.hip)
    if (max_own <= 64 && max_obs <= 48 && !std::getenv("SFM_BA_TILE80")) {
        // both tile heights are planned concurrently (independent, read-only inputs)
        std::vector<ChunkDesc> c4, c5;
        std::vector<int32_t> s4, s5;
        int64_t f4 = 0, f5 = 0;
        int rc5 = SFM_OK;
        std::thread t5([&] {
            rc5 = guarded([&] {
                f5 = make_chunks(kTileRowsUsed, c5, s5);
                return SFM_OK;
            });
        });
        int rc4 = guarded([&] {
            f4 = make_chunks(64, c4, s4);
            return SFM_OK;
        });
        t5.join();
        if (rc4 != SFM_OK) throw SfmError{rc4};
        if (rc5 != SFM_OK) throw SfmError{rc5};
        if (c4.size() * 4 <= c5.size() * 5) {
            pl.tile_nt = 4; pl.chunks.swap(c4); pl.obs_slot.swap(s4); flops = f4;
        } else {
            pl.chunks.swap(c5); pl.obs_slot.swap(s5); flops = f5;
        }
    } else {
        flops = make_chunks(kTileRowsUsed, pl.chunks, pl.obs_slot);
    }
    pl.schur_flops = flops;
    pl.schur_bytes = pl.n_sobs * (16 + 4 + 4 + 4) + pl.n_spt * (24 + 24 + 4) +
                     (int64_t)pl.chunks.size() * kTileR * kTileR * 8;

    // ---- image CSR of shard observations ------------------------------------
    // counting sort by image, in parallel: per-range counts, then each range
    // scatters from its own offsets (ranges in order => shard order per image)
    pl.img_obs_ptr.assign(P.n_img + 1, 0);
    pl.img_obs.resize(pl.n_sobs);
    pl.img_pt.resize(pl.n_sobs);
    pl.img_uv.resize(2 * pl.n_sobs);
    {
        constexpr int kMaxT = 16;
        std::vector<std::vector<int32_t>> cnt(kMaxT);
        std::vector<std::pair<int64_t, int64_t>> rng(kMaxT, {0, 0});
        parallel_ranges(pl.n_sobs, [&](int64_t s0, int64_t s1, int t) {
            rng[t] = {s0, s1};
            cnt[t].assign(P.n_img, 0);
            for (int64_t s = s0; s < s1; ++s) cnt[t][pl.obs_img[s]]++;
        });
        for (int i = 0; i < P.n_img; ++i) {
            int32_t tot = 0;
            for (int t = 0; t < kMaxT; ++t)
                if (!cnt[t].empty()) tot += cnt[t][i];
            pl.img_obs_ptr[i + 1] = pl.img_obs_ptr[i] + tot;
        }
        // per-range write cursors: image start + counts of earlier ranges
        for (int i = 0; i < P.n_img; ++i) {
            int32_t at = pl.img_obs_ptr[i];
            for (int t = 0; t < kMaxT; ++t)
                if (!cnt[t].empty()) {
                    const int32_t c = cnt[t][i];
                    cnt[t][i] = at;
                    at += c;
                }
        }
        parallel_ranges(pl.n_sobs, [&](int64_t s0, int64_t s1, int t) {
            std::vector<int32_t>& fill = cnt[t];
            for (int64_t s = s0; s < s1; ++s) {
                const int32_t q = fill[pl.obs_img[s]]++;
                pl.img_obs[q] = (int32_t)s;
                pl.img_pt[q] = pl.obs_pt[s];
                pl.img_uv[2 * q] = pl.obs_uv[2 * s];
                pl.img_uv[2 * q + 1] = pl.obs_uv[2 * s + 1];
            }
        });
    }

    // ---- reduce plan -----------------------------------------------------------
    const int Dp = pl.D + 1;
    pl.n_sband = (int64_t)pl.ncam * Dp * 36;
    pl.n_sarrow = (int64_t)pl.nintr * pl.ncam * 24;
    pl.n_scorner = (int64_t)pl.nintr * pl.nintr * 16;
    // chunk slot lookups: block -> (chunk, row)
    std::map<int64_t, std::vector<ReduceTerm>> band, arrow, corner, rhs;  // keyed by target
    for (int32_t c = 0; c < (int32_t)pl.chunks.size(); ++c) {
        const ChunkDesc& cd = pl.chunks[c];
        for (int a = 0; a < cd.n_slots; ++a) {
            // rhs contribution (-Z w) from tile row 79
            rhs[cd.slot_col[a]].push_back(ReduceTerm{kSrcTile, c, (int16_t)kTileWRow, (int16_t)cd.slot_row[a], 1.f});
            for (int b = 0; b < cd.n_slots; ++b) {
                const bool ac = cd.slot_img[a] >= 0, bc = cd.slot_img[b] >= 0;
                if (ac && bc) {
                    const int ia = pl.cam_blk[cd.slot_img[a]], ib = pl.cam_blk[cd.slot_img[b]];
                    if (ia < ib) continue;
                    band[(int64_t)ia * Dp + (ia - ib)].push_back(
                        ReduceTerm{kSrcTile, c, (int16_t)cd.slot_row[a], (int16_t)cd.slot_row[b], 1.f});
                } else if (!ac && bc) {
                    const int k = pl.intr_blk[cd.slot_intr[a]], ib = pl.cam_blk[cd.slot_img[b]];
                    arrow[(int64_t)k * pl.ncam + ib].push_back(
                        ReduceTerm{kSrcTile, c, (int16_t)cd.slot_row[a], (int16_t)cd.slot_row[b], 1.f});
                } else if (!ac && !bc) {
                    const int k = pl.intr_blk[cd.slot_intr[a]], l = pl.intr_blk[cd.slot_intr[b]];
                    corner[(int64_t)k * pl.nintr + l].push_back(
                        ReduceTerm{kSrcTile, c, (int16_t)cd.slot_row[a], (int16_t)cd.slot_row[b], 1.f});
                }
            }
        }
    }
    auto emit = [&](int32_t kind, int64_t dst, int rows, int cols, int ld, std::vector<ReduceTerm>* tl,
                    std::vector<ReduceTerm> extra) {
        ReduceTarget t{};
        t.dst = dst; t.dst_kind = kind; t.rows = rows; t.cols = cols; t.ld = ld;
        t.c_begin = (int32_t)pl.terms.size();
        for (const auto& e : extra)   // image Gram blocks come in kGramSeg partial slices
            for (int g = 0; g < (e.kind == kSrcTile ? 1 : kGramSeg); ++g) {
                ReduceTerm q = e;
                if (e.kind != kSrcTile) q.index = e.index * kGramSeg + g;
                pl.terms.push_back(q);
            }
        if (tl) for (const auto& e : *tl) pl.terms.push_back(e);
        t.c_end = (int32_t)pl.terms.size();
        pl.targets.push_back(t);
    };
    for (int i = 0; i < pl.ncam; ++i) {
        const int img = pl.blk_img[i];
        for (int d = 0; d <= std::min(pl.D, i); ++d) {
            auto it = band.find((int64_t)i * Dp + d);
            std::vector<ReduceTerm> ex;
            if (d == 0) ex.push_back(ReduceTerm{kSrcU, img, 0, 0, 1.f});
            emit(0, ((int64_t)i * Dp + d) * 36, 6, 6, 6, it == band.end() ? nullptr : &it->second, ex);
        }
    }
    for (int k = 0; k < pl.nintr; ++k)
        for (int i = 0; i < pl.ncam; ++i) {
            const int img = pl.blk_img[i];
            auto it = arrow.find((int64_t)k * pl.ncam + i);
            std::vector<ReduceTerm> ex;
            if (pl.intr_blk[P.img_intr[img]] == k) ex.push_back(ReduceTerm{kSrcU, img, 6, 0, 1.f});
            emit(1, ((int64_t)k * pl.ncam + i) * 24, 4, 6, 6, it == arrow.end() ? nullptr : &it->second, ex);
        }
    for (int k = 0; k < pl.nintr; ++k)
        for (int l = 0; l < pl.nintr; ++l) {
            auto it = corner.find((int64_t)k * pl.nintr + l);
            std::vector<ReduceTerm> ex;
            if (k == l)
                for (int img = 0; img < P.n_img; ++img)
                    if (pl.intr_blk[P.img_intr[img]] == k) ex.push_back(ReduceTerm{kSrcU, img, 6, 6, 1.f});
            emit(2, ((int64_t)k * pl.nintr + l) * 16, 4, 4, 4, it == corner.end() ? nullptr : &it->second, ex);
        }
    // vectors: rhs = bF - Z w, bF, cnF
    for (int vk = 3; vk <= 5; ++vk) {
        for (int i = 0; i < pl.ncam; ++i) {
            const int img = pl.blk_img[i];
            std::vector<ReduceTerm> ex{ReduceTerm{vk == 5 ? kSrcUcn : kSrcUb, img, 0, 0, 1.f}};
            auto it = rhs.find(6LL * i);
            emit(vk, 6LL * i, 6, 1, 1, (vk == 3 && it != rhs.end()) ? &it->second : nullptr, ex);
        }
        for (int k = 0; k < pl.nintr; ++k) {
            std::vector<ReduceTerm> ex;
            for (int img = 0; img < P.n_img; ++img)
                if (pl.intr_blk[P.img_intr[img]] == k)
                    ex.push_back(ReduceTerm{vk == 5 ? kSrcUcn : kSrcUb, img, 6, 0, 1.f});
            auto it = rhs.find(pl.nb + 4LL * k);
            emit(vk, pl.nb + 4LL * k, 4, 1, 1, (vk == 3 && it != rhs.end()) ? &it->second : nullptr, ex);
        }
    }
}

}  // namespace sfm

extern "C" int sfm_ba_partition(const sfm_ba_problem* prob, int32_t world_size, int64_t* order,
                                int64_t* bounds) {
    using namespace sfm;
    return guarded([&] {
        SFM_REQUIRE(prob && order && bounds && world_size >= 1, SFM_ERR_INVALID_ARG, "bad arguments");
        BAHostPlan tmp;
        std::vector<int32_t> cam_blk(prob->n_img, -1);
        int nc = 0;
        std::vector<char> used(prob->n_img, 0);
        for (int64_t o = 0; o < prob->n_obs; ++o) used[prob->obs_img[o]] = 1;
        for (int i = 0; i < prob->n_img; ++i)
            if (used[i] && i != prob->const_img) cam_blk[i] = nc++;
        std::vector<int64_t> ord, bnd;
        partition_points(*prob, cam_blk, world_size, ord, bnd);
        std::copy(ord.begin(), ord.end(), order);
        std::copy(bnd.begin(), bnd.end(), bounds);
        return SFM_OK;
    });
}
