// Block cyclic reduction solve of the reduced camera system (ba_bcr.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "ba_kernels.h"

namespace sfm {

constexpr int kBcrM = 64;   // super-block size (scalars)
constexpr int kBcrK = 10;   // camera blocks per super-block (6*K <= 64)

struct BcrArgs {
    int N = 0;      // super-blocks
    int K = 0;      // camera blocks per super-block
    int nrhs = 0;   // 1 + iw*nintr (rhs + arrow columns), padded to a multiple of 16
    double *A = nullptr, *C = nullptr, *L = nullptr, *Wl = nullptr, *Wr = nullptr;
    // R: rhs + arrow columns as updated; Z: each block's forward solve X R;
    // Y: the back substitution's y, as 128 tagged granules per block; part: corner partials;
    // fail: [0] numerical, [1] wait timeout, [4] / [6] corner tickets, [5] back-substitution ticket
    double *R = nullptr, *Z = nullptr, *Y = nullptr, *part = nullptr, *fail = nullptr;
    unsigned* yflag = nullptr;   // [N] back substitution: y_i published for epoch (bcr_back_kernel<true>)
    unsigned long long* stamps = nullptr;   // SFM_BCR_STAMPS diagnostic: phase cycle sums
    bool split = false;   // SFM_CTX_BA_SPLIT_BCR: top, corner and each back-substitution level as own launches
};

// Dense RCS solve (blocked Cholesky on 64x64 tiles, same file).
struct DenseArgs {
    int nt = 0;          // tiles per side
    int64_t np = 0;      // padded order nt * 64
    double *A = nullptr, *X = nullptr, *b = nullptr, *y = nullptr, *x = nullptr, *fail = nullptr;
    unsigned* xflag = nullptr;   // [nt] back substitution: x_k published for epoch (dense_back_all_kernel)
    unsigned* fflag = nullptr;   // [2 nt^2 + nt] dataflow factorisation: L tiles, chain inputs, y (dense_flow_kernel)
    unsigned long long* xg = nullptr;   // [nt][kYG] dataflow back substitution: x_k as tagged granules
    unsigned long long* stamps = nullptr;   // SFM_DENSE_STAMPS diagnostic: chain phase sums, real-time spans
    // dataflow solve (dense_flow_kernel, nt <= kDenseFlowMaxNt): the host's
    // schedule (dense_flow_plan): tile order, chains, tile pattern, task list
    const int32_t* meta = nullptr;
    int nch = 0, ntask = 0;    // chain workgroups (1 or 2), tasks
    int64_t meta_words = 0;    // int32 words at meta
    bool flow = false;         // the dataflow kernel solves (else the launch chain)
    bool chain = false;   // SFM_CTX_BA_DENSE_CHAIN: launch chains instead of the dataflow kernels
};
// flag words of a DenseArgs (x flags + the factorisation's + the x granules), zeroed once at bind
size_t dense_flag_words(const DenseArgs& d);
void dense_setup(DenseArgs& d, const DevProblem& P);
// the dataflow solve's schedule (host, once per plan; empty for the launch
// chain): sets d.flow / nch / ntask / meta_words; the caller copies it to d.meta
// exact: the natural tiles' coupling from the reduce targets (dense_tile_pattern),
// used to order the tiles when the intrinsics arrow is itself banded
std::vector<int32_t> dense_flow_plan(DenseArgs& d, const DevProblem& P, const std::vector<char>* exact = nullptr);
// tile (a, b), a >= b, of the natural order is nonzero: some dense reduce
// target touches it, or a == b ([nt][nt] bytes, lower triangle)
std::vector<char> dense_tile_pattern(const std::vector<ReduceTarget>& targets, int64_t nF, int nt);
size_t dense_doubles(const DenseArgs& d);
void dense_bind(DenseArgs& d, double* base);
// epoch: a value the x flags do not hold yet (the plan counts its solves from 1)
void dense_solve(const DenseArgs& d, const DevProblem& P, double radius, hipStream_t s, unsigned epoch);

bool bcr_supported(const DevProblem& P);
void bcr_setup(BcrArgs& b, const DevProblem& P);
size_t bcr_doubles(const BcrArgs& b);
// 8-byte words of the back substitution's tagged y granules at b.Y (zeroed once at bind)
inline size_t bcr_y_granules(const BcrArgs& b) { return (size_t)b.N * 128; }
void bcr_bind(BcrArgs& b, double* base);
// The LM candidate, formed by the back substitution as each block's y is
// known (cand_kernel's arithmetic, ba_cand.h): the current point's extrinsics
// and intrinsics, and the candidate's extrinsics, intrinsics and CamPre
struct BcrCand {
    const double* extr;
    const double* intr;
    double* cand_extr;
    double* cand_intr;
    CamPre* cand_cp;
};
// epoch: a value the y granules do not hold yet (the plan counts its solves from 1)
void bcr_solve(const BcrArgs& b, const DevProblem& P, double radius, hipStream_t s, unsigned epoch,
               const BcrCand& cand);

}  // namespace sfm
