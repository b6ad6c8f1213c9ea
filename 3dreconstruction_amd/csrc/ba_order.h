// Device-side planning helpers (ba_order.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"

namespace sfm {

// Image order of a shard's observations (stable by image, shard order within
// one): img_pt[q] = owning shard point, img_uv[2q..] = measurement.  Inputs
// and outputs are device arrays; runs on stream s.
void ba_image_order(const int32_t* obs_img, const double* obs_uv, const int32_t* pt_off, int32_t n_sobs,
                    int32_t n_spt, int32_t n_img, int32_t* img_pt, double* img_uv, hipStream_t s);

// Refresh of a cached plan with new values (sfm_ba_solve's plan cache):
// obs_src[s] = the problem observation of shard observation s; then the
// measurements and points gathered into shard order on the device.
void ba_obs_source(const int32_t* pt_src, const int64_t* pt_offsets, const int32_t* pt_off, int32_t n_spt,
                   int32_t n_cpt, const int32_t* gperm, int32_t* obs_src, hipStream_t s);
void ba_gather_uv(const int32_t* obs_src, const double* src_uv, int32_t n_sobs, double* dst_uv, hipStream_t s);
void ba_gather_points(const int32_t* pt_src, const double* src_X, int32_t n_spt, double* dst_X, hipStream_t s);

}  // namespace sfm
