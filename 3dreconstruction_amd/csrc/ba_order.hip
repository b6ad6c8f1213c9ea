// Device-side part of BA planning: the image-ordered copy of a shard's
// observations that the image Gram pass (image_gram_kernel) walks.
//
// The host planner used to build it with a counting sort and upload three
// more observation-sized arrays (120 MB at C4); here the observations already
// resident in HBM are stably radix-sorted by image (rocPRIM through hipCUB:
// shard order is kept within an image, the order the host sort produced) and
// the point index and measurement gathered in that order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "ba_order.h"

namespace sfm {
namespace {

// obs_pt[s] = the shard point owning observation s
__global__ __launch_bounds__(256) void obs_point_kernel(const int32_t* __restrict__ pt_off, int32_t n_spt,
                                                        int32_t* __restrict__ obs_pt) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n_spt) return;
    for (int s = pt_off[k]; s < pt_off[k + 1]; ++s) obs_pt[s] = k;
}

__global__ __launch_bounds__(256) void iota_kernel(int32_t* __restrict__ v, int32_t n) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s < n) v[s] = s;
}

// image order: point and measurement of the observation at each position
__global__ __launch_bounds__(256) void image_gather_kernel(const int32_t* __restrict__ order,
                                                           const int32_t* __restrict__ obs_pt,
                                                           const double2* __restrict__ obs_uv, int32_t n,
                                                           int32_t* __restrict__ img_pt, double2* __restrict__ img_uv) {
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const int s = order[q];
    img_pt[q] = obs_pt[s];
    img_uv[q] = obs_uv[s];
}

}  // namespace

void ba_image_order(const int32_t* obs_img, const double* obs_uv, const int32_t* pt_off, int32_t n_sobs,
                    int32_t n_spt, int32_t n_img, int32_t* img_pt, double* img_uv, hipStream_t s) {
    if (n_sobs <= 0) return;
    DBuf<int32_t> obs_pt, idx, order, keys_out;
    obs_pt.alloc(n_sobs);
    idx.alloc(n_sobs);
    order.alloc(n_sobs);
    keys_out.alloc(n_sobs);
    const unsigned gs = (unsigned)((n_sobs + 255) / 256);
    hipLaunchKernelGGL(obs_point_kernel, dim3((unsigned)((n_spt + 255) / 256)), dim3(256), 0, s, pt_off, n_spt,
                       obs_pt.p);
    SFM_HIP(hipGetLastError());
    hipLaunchKernelGGL(iota_kernel, dim3(gs), dim3(256), 0, s, idx.p, n_sobs);
    SFM_HIP(hipGetLastError());
    int end_bit = 1;
    while (end_bit < 31 && (1 << end_bit) < n_img) ++end_bit;
    size_t tmp_bytes = 0;
    SFM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, obs_img, keys_out.p, idx.p, order.p, n_sobs, 0,
                                               end_bit, s));
    DBuf<uint8_t> tmp;
    tmp.alloc(std::max<size_t>(tmp_bytes, 1));
    SFM_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tmp_bytes, obs_img, keys_out.p, idx.p, order.p, n_sobs, 0,
                                               end_bit, s));
    hipLaunchKernelGGL(image_gather_kernel, dim3(gs), dim3(256), 0, s, order.p, obs_pt.p,
                       reinterpret_cast<const double2*>(obs_uv), n_sobs, img_pt, reinterpret_cast<double2*>(img_uv));
    SFM_HIP(hipGetLastError());
    // the temporaries go back to the context's cache, stream-ordered
}

namespace {

// shard observation s of shard point k: source observation pt_offsets[pt_src[k]] + (s - pt_off[k]) for
// a point that kept the problem's order; a general point re-sorted by image (k >= n_cpt) maps through
// gperm[s - pt_off[n_cpt]] (null: no point was re-sorted)
__global__ void obs_source_kernel(const int32_t* __restrict__ pt_src, const int64_t* __restrict__ pt_offsets,
                                  const int32_t* __restrict__ pt_off, int32_t n_spt, int32_t n_cpt,
                                  const int32_t* __restrict__ gperm, int32_t* __restrict__ obs_src) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_spt) return;
    const int64_t o0 = pt_offsets[pt_src[k]];
    if (gperm && k >= n_cpt) {
        const int32_t g0 = pt_off[n_cpt];
        for (int32_t s = pt_off[k]; s < pt_off[k + 1]; ++s) obs_src[s] = (int32_t)(o0 + gperm[s - g0]);
    } else {
        for (int32_t s = pt_off[k]; s < pt_off[k + 1]; ++s) obs_src[s] = (int32_t)(o0 + (s - pt_off[k]));
    }
}

__global__ void gather_uv_kernel(const int32_t* __restrict__ obs_src, const double2* __restrict__ src, int32_t n,
                                 double2* __restrict__ dst) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) dst[s] = src[obs_src[s]];
}

__global__ void gather_points_kernel(const int32_t* __restrict__ pt_src, const double* __restrict__ src, int32_t n,
                                     double* __restrict__ dst) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= 3 * n) return;
    const int k = e / 3;
    dst[e] = src[3 * (int64_t)pt_src[k] + (e - 3 * k)];
}

}  // namespace

void ba_obs_source(const int32_t* pt_src, const int64_t* pt_offsets, const int32_t* pt_off, int32_t n_spt,
                   int32_t n_cpt, const int32_t* gperm, int32_t* obs_src, hipStream_t s) {
    if (n_spt <= 0) return;
    hipLaunchKernelGGL(obs_source_kernel, dim3((unsigned)((n_spt + 255) / 256)), dim3(256), 0, s, pt_src, pt_offsets,
                       pt_off, n_spt, n_cpt, gperm, obs_src);
    SFM_HIP(hipGetLastError());
}

void ba_gather_uv(const int32_t* obs_src, const double* src_uv, int32_t n_sobs, double* dst_uv, hipStream_t s) {
    if (n_sobs <= 0) return;
    hipLaunchKernelGGL(gather_uv_kernel, dim3((unsigned)((n_sobs + 255) / 256)), dim3(256), 0, s, obs_src,
                       reinterpret_cast<const double2*>(src_uv), n_sobs, reinterpret_cast<double2*>(dst_uv));
    SFM_HIP(hipGetLastError());
}

void ba_gather_points(const int32_t* pt_src, const double* src_X, int32_t n_spt, double* dst_X, hipStream_t s) {
    if (n_spt <= 0) return;
    hipLaunchKernelGGL(gather_points_kernel, dim3((unsigned)((3 * (int64_t)n_spt + 255) / 256)), dim3(256), 0, s,
                       pt_src, src_X, n_spt, dst_X);
    SFM_HIP(hipGetLastError());
}

}  // namespace sfm
