// Types shared by the BA host planner (ba_plan.cpp), the LM driver
// (ba_solver.cpp) and the gfx950 kernels (ba_kernels.hip).
//
// HBM layout (DESIGN.md §BA data layout), per rank:
//   points   : X[3*n_spt] in shard order (landmark-major, sorted by first
//              active camera), scaleE[3*n_spt] (Jacobi scale, fixed at iter 0)
//   obs      : obs_uv[2*n_sobs], obs_img[n_sobs], pt_off[n_spt+1]
//              (observations of a point contiguous)
//   cameras  : extr[6*n_img], intr[4*n_intr] (full tables, replicated),
//              CamPre[n_img] (per-camera rotation terms), scaleF[nF]
//   RCS      : Sband[ncam][D+1][6][6] (block (i,i-d)), Sarrow[nintr][ncam][4][6],
//              Scorner[nintr][nintr][4][4], rhs[nF], bF[nF], cnF[nF]
//   chunk slab: tiles[n_group][80][80] (-Z Z^T, row 79 = -Z w), one per tile group of <= 4 chunks
//   image slab: Uimg[n_img][FW][FW], Ub[n_img][FW], Ucn[n_img][FW] (FW = 6 + intrinsics width)
#pragma once
#include <cstdint>

namespace sfm {

constexpr int kTileN = 5;                 // 16-row MFMA tiles per chunk side
constexpr int kTileR = 16 * kTileN;       // 80 rows
constexpr int kTileRowsUsed = 76;         // rows 0..75 for F blocks
constexpr int kTileWRow = 79;             // row carrying w = L^-1 g_E
constexpr int kSubPts = 6;                // points per wave batch (3 panel columns each)
constexpr int kZShortObs = 32;            // general points the batched Z kernel takes (observations)
constexpr int kZBatchPts = 16;            // points per batch of that kernel
constexpr int kSubObs = 64;               // observations per wave batch (one per lane)
// points / observations per batch of the 64-row Schur variant, by residual
// model (SFM_CAM_*: 0 pinhole, 1 BAL, 2 RADIAL3), sized so its LDS stays
// under 20 KB, i.e. 8 waves per CU (the register limit): pinhole 5 / 52
// (20.2 KB), BAL 4 / 48 (17.8 KB; 5 points would pass 20 KB), RADIAL3 4 / 44
// (19.4 KB; 48 observations: 20.1 KB, 7 waves).  A point above the
// observation count goes to the 80-row variant.
constexpr int schur4_pts(int cm) { return cm == 0 ? 5 : 4; }
constexpr int schur4_obs(int cm) { return cm == 0 ? 52 : cm == 2 ? 44 : 48; }
constexpr int kChunkPts = 128;            // points per chunk (upper bound; step_kernel threads)
constexpr int kGroupChunks = 4;           // chunks per tile group, at most (the Schur kernel's waves per workgroup)
// chunks per tile group by tile height: 4 for 64-row tiles (four waves' LDS
// is 60-68 KB: two workgroups, 8 waves per CU as one-wave chunks had), 1 for
// 80-row tiles (their 26-30 KB per wave: two-wave groups would cost the
// RADIAL3 variant a wave per CU)
// Default 1 (round 4): four-chunk groups cut the tile writes four-fold and
// the reduce kernels from 39 to 27 us per iteration at C4, but the Schur
// launch went 0.339 -> 0.368 ms (a group's waves finish together and hold
// its LDS until the slowest is done): C4 1041 vs 1048 LM-iters/s on one box
// (profiles/r04/c_jit/ab.txt).  The group machinery stays (a group of one
// chunk is the shipped form); the grouped form was an A/B build, not kept.
constexpr int schur_group(int) { return 1; }
constexpr int kGramSeg = 3;   // workgroups per image in the image Gram pass (at most)
constexpr int kMaxSlots = 16;             // F slots (row-carrying cameras + intrinsics)
constexpr int kCamSlots = 14;             // staged cameras per chunk (incl. constant images)
constexpr int kIntrSlots = 4;             // staged intrinsics blocks per chunk
constexpr int kZMaxDoubles = 18432;       // LDS Z accumulator of one general point (144 KB):
                                          // ~1000 parameter blocks per point

// Per-camera precomputed rotation terms (for current or candidate params).
//   Rodrigues branch: P = X c + (u x X) s + u (u.X)(1-c) + t,
//                     dP/dX = R, dP/dw = -R [X]x Ar  (Ar = (w w' + (R'-I)[w]x)/|w|^2)
//   small-angle branch (|w|^2 <= eps): P = X + w x X + t, dP/dX = I + [w]x,
//                     dP/dw = -[X]x (R := I + [w]x for dP/dX, left factor I, Ar = I)
struct alignas(16) CamPre {
    double c, s, omc, small;   // cos, sin, 1-cos, small-angle flag (0/1)
    double u[3];               // unit axis (Rodrigues) or w (small angle)
    double t[3];
    double R[9];               // dP/dX; left factor of dP/dw is R (Rodrigues) or I (small)
    double Ar[9];              // right factor of dP/dw
};

// obs_slot of an observation: staged camera index | (staged intrinsics index << 8)
struct ChunkDesc {
    int32_t pt_begin, pt_end;      // shard point range
    int32_t obs_begin, obs_end;    // shard obs range
    int32_t n_slots;               // F slots (reduce plan)
    int32_t n_cams, n_intr;        // staged cameras / intrinsics
    int32_t sub;                   // index within its tile group (the group's slot layout)
    int32_t cam_img[kCamSlots];    // image of a staged camera
    int32_t cam_row[kCamSlots];    // its first tile row, -1 for a constant image
    int32_t cam_col[kCamSlots];    // its first scaleF column, -1 for a constant image
    int32_t intr_id[kIntrSlots];   // staged intrinsics block
    int32_t intr_row[kIntrSlots];  // its first tile row
    int32_t intr_col[kIntrSlots];  // its first scaleF column
    int32_t slot_img[kMaxSlots];   // image of a camera slot (or -1)
    int32_t slot_intr[kMaxSlots];  // intrinsic block of an intr slot (or -1)
    int32_t slot_row[kMaxSlots];   // first tile row of the slot
    int32_t slot_col[kMaxSlots];   // global F column of the slot
};

// Reduce-plan term sources (kind).
enum : int32_t { kSrcTile = 0, kSrcU = 1, kSrcUb = 2, kSrcUcn = 3 };

struct ReduceTarget {
    int64_t dst;        // element offset of the block in its destination array
    int32_t dst_kind;   // 0 Sband, 1 Sarrow, 2 Scorner, 3 rhs, 4 bF, 5 cnF, 6 Sdense
    int32_t rows, cols; // block shape (vectors: cols = 1)
    int32_t ld;         // destination row stride
    int32_t c_begin, c_end;  // sum-term range (chunk tiles, image Gram blocks)
    int32_t p_begin, p_end;  // product-term range (general points, PTerm)
};

// Product term of a general point (one not handled by a Schur chunk): the
// target block gets -Z_a Z_b' (rows x cols, inner dimension 3), Z_a and Z_b
// the point's eliminated rows of blocks a and b, row-major [rows][3] at
// element offsets za / zb of the Z buffer; for a vector target Z_b is the
// point's w = L^-1 g_E (one row of 3).  32-bit offsets (the planner requires
// a Z buffer under 2^31 doubles): half the bytes the planner writes and the
// reduce reads per term (round 6).
struct PTerm {
    int32_t za, zb;
};

// Kinds of dst_kind.
enum : int32_t { kDstBand = 0, kDstArrow = 1, kDstCorner = 2, kDstRhs = 3, kDstBF = 4, kDstCnF = 5,
                 kDstDense = 6 };

// ReduceTerm resolved against the contiguous [tiles | U | Ub | Ucn] buffer.
// Chunk tiles hold only their lower 16x16 tiles (diagonal tiles whole), so a
// tile block is read in one of three modes:
//   kFlatRows  element (r, c) at src[off + r * rs + c]       (lower blocks, U, vectors)
//   kFlatTrans element (r, c) at src[off + c * kTileR + r]   (upper blocks: the
//              symmetric partner; off addresses the partner's origin)
//   kFlatSym   element (r, c) of a diagonal slot block: tile position
//              (R, C) = origin + (r, c) read at (max, min); off addresses
//              the origin, rs holds its offset within the chunk tile
enum : int16_t { kFlatRows = 0, kFlatTrans = 1, kFlatSym = 2 };
struct FlatTerm {
    int64_t off;
    int16_t rs;
    int16_t mode;
    float sign;
};

struct ReduceTerm {
    int32_t kind;       // kSrc*
    int32_t index;      // chunk or image
    int16_t roff, coff; // source block origin
    float sign;         // +1 / -1
};

}  // namespace sfm
