/*
 * vlsift_tool — golden-descriptor generator (TEST INFRASTRUCTURE ONLY).
 *
 * Links the reference's in-tree VLFeat (src/nonFree/sift/vl/*.c, compiled in
 * place by oracle/build_ref.sh into oracle/_ref/) and reproduces the
 * descriptor path of SIFT_Image_describer::DescribeSIFT
 * (src/nonFree/sift/SIFT_describer.hpp:141-220) with the default Params
 * (:55-68: first octave 0, 6 octaves, 3 scales, edge 10, peak 0.04,
 * RootSIFT) and siftDescToUChar (:31-45).  Input images are synthetic and
 * deterministic (blob field rendered under an affine warp), so two views
 * share true correspondences.
 *
 * usage: vlsift_tool <out.u8> <out.kp> <width> <height> <seed> <angle> <tx> <ty> <scale>
 *   out.u8: n x 128 uchar descriptors; out.kp: n x 4 float (x, y, sigma, angle)
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "sift.h"
#include "generic.h"

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static double uni(uint64_t seed, uint64_t k) { return (double)(mix64(seed + 0x9E3779B97F4A7C15ULL * (k + 1)) >> 11) * 0x1.0p-53; }

#define NBLOB 900
static double bx[NBLOB], by[NBLOB], bs[NBLOB], ba[NBLOB], be[NBLOB];

static double field(double x, double y) {
    double v = 110.0;
    for (int i = 0; i < NBLOB; ++i) {
        const double dx = x - bx[i], dy = y - by[i];
        const double r2 = (dx * dx + be[i] * dy * dy) / (bs[i] * bs[i]);
        if (r2 < 16.0) v += ba[i] * exp(-0.5 * r2);
    }
    return v < 0 ? 0 : (v > 255 ? 255 : v);
}

int main(int argc, char** argv) {
    if (argc != 10) { fprintf(stderr, "usage: %s out.u8 out.kp w h seed angle tx ty scale\n", argv[0]); return 2; }
    const int w = atoi(argv[3]), h = atoi(argv[4]);
    const uint64_t seed = strtoull(argv[5], 0, 0);
    const double ang = atof(argv[6]), tx = atof(argv[7]), ty = atof(argv[8]), sc = atof(argv[9]);
    for (int i = 0; i < NBLOB; ++i) {
        bx[i] = uni(seed, 5 * i) * w * 1.2 - 0.1 * w;
        by[i] = uni(seed, 5 * i + 1) * h * 1.2 - 0.1 * h;
        bs[i] = 2.0 + 14.0 * uni(seed, 5 * i + 2);
        ba[i] = (uni(seed, 5 * i + 3) - 0.5) * 220.0;
        be[i] = 0.4 + 1.6 * uni(seed, 5 * i + 4);
    }
    /* image(u, v) = field(A^-1 ((u, v) - c) + c - t): a rotated/scaled/shifted view */
    float* img = (float*)malloc(sizeof(float) * w * h);
    const double ca = cos(ang) / sc, sa = sin(ang) / sc, cx = 0.5 * w, cy = 0.5 * h;
    for (int v = 0; v < h; ++v)
        for (int u = 0; u < w; ++u) {
            const double du = u - cx - tx, dv = v - cy - ty;
            const double x = ca * du + sa * dv + cx, y = -sa * du + ca * dv + cy;
            /* uchar quantisation as the reference's image::Image<unsigned char> input */
            img[v * w + u] = (float)(unsigned char)(field(x, y) + 0.5);
        }

    vl_constructor();
    VlSiftFilt* filt = vl_sift_new(w, h, 6, 3, 0);
    vl_sift_set_edge_thresh(filt, 10.0f);
    vl_sift_set_peak_thresh(filt, 255 * 0.04f / 3);
    FILE* fd = fopen(argv[1], "wb");
    FILE* fk = fopen(argv[2], "wb");
    long n = 0;
    if (vl_sift_process_first_octave(filt, img) != VL_ERR_EOF) {
        while (1) {
            vl_sift_detect(filt);
            const VlSiftKeypoint* keys = vl_sift_get_keypoints(filt);
            const int nkeys = vl_sift_get_nkeypoints(filt);
            vl_sift_update_gradient(filt);
            for (int i = 0; i < nkeys; ++i) {
                double angles[4];
                const int na = vl_sift_calc_keypoint_orientations(filt, angles, keys + i);
                for (int q = 0; q < na; ++q) {
                    vl_sift_pix d[128];
                    vl_sift_calc_keypoint_descriptor(filt, d, keys + i, angles[q]);
                    float sum = 0.f;
                    for (int k = 0; k < 128; ++k) sum += d[k];
                    unsigned char u8[128];
                    for (int k = 0; k < 128; ++k) u8[k] = (unsigned char)(512.f * sqrtf(d[k] / sum));
                    const float kp[4] = {keys[i].x, keys[i].y, keys[i].sigma, (float)angles[q]};
                    fwrite(u8, 1, 128, fd);
                    fwrite(kp, sizeof(float), 4, fk);
                    ++n;
                }
            }
            if (vl_sift_process_next_octave(filt)) break;
        }
    }
    fclose(fd);
    fclose(fk);
    vl_sift_delete(filt);
    vl_destructor();
    free(img);
    printf("%ld\n", n);
    return 0;
}
