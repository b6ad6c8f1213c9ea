// Minimal data model with the reference's shape (no OpenCV/Eigen/Sophus/PCL):
//   Camera       src/component/Camera.h:11-100  (fx, fy, cx, cy; getIntrinsic/setIntrinsic)
//   Image        src/component/Image.h:16-151   (Tcw pose as angle-axis + t, descriptors,
//                                                keypoints, keypoint -> world point map)
//   WorldPoint   src/world/WorldPoint.h:13-41   (world_pos_, last_descriptor_, observed_frames_)
//   WorldStructure src/world/WorldStructure.h:70-99 (local_frames_, images_, world_points_)
//   LocalFrame   src/frame/LocalFrame.h:19-83   (image pair + matches)
// The fields BundleAdjuster and the matchers read/write keep their names.
#pragma once
#include <algorithm>
#include <array>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <unordered_map>
#include <utility>
#include <vector>

namespace sfm {

struct Point2d {
    double x = 0, y = 0;
};

struct DMatch {            // cv::DMatch subset
    int queryIdx = -1, trainIdx = -1, imgIdx = 0;
    float distance = 0.f;  // sqrt of the exact squared L2
};

// Rotation helpers (angle-axis <-> matrix, ZYX Euler) for pose marshalling.
namespace rot {
inline void aa_to_matrix(const double w[3], double R[9]) {
    const double th = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    if (th < 1e-300) {
        for (int a = 0; a < 9; ++a) R[a] = (a % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    const double u[3] = {w[0] / th, w[1] / th, w[2] / th}, c = std::cos(th), s = std::sin(th), oc = 1 - c;
    R[0] = c + oc * u[0] * u[0];        R[1] = oc * u[0] * u[1] - s * u[2]; R[2] = oc * u[0] * u[2] + s * u[1];
    R[3] = oc * u[1] * u[0] + s * u[2]; R[4] = c + oc * u[1] * u[1];        R[5] = oc * u[1] * u[2] - s * u[0];
    R[6] = oc * u[2] * u[0] - s * u[1]; R[7] = oc * u[2] * u[1] + s * u[0]; R[8] = c + oc * u[2] * u[2];
}
inline void matrix_to_aa(const double R[9], double w[3]) {
    const double tr = R[0] + R[4] + R[8];
    double q[4];
    if (tr >= 0) {
        double t = std::sqrt(tr + 1.0);
        q[0] = 0.5 * t; t = 0.5 / t;
        q[1] = (R[7] - R[5]) * t; q[2] = (R[2] - R[6]) * t; q[3] = (R[3] - R[1]) * t;
    } else {
        int i = 0;
        if (R[4] > R[0]) i = 1;
        if (R[8] > R[i * 4]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double t = std::sqrt(R[i * 4] - R[j * 4] - R[k * 4] + 1.0);
        q[i + 1] = 0.5 * t; t = 0.5 / t;
        q[0] = (R[k * 3 + j] - R[j * 3 + k]) * t;
        q[j + 1] = (R[j * 3 + i] + R[i * 3 + j]) * t;
        q[k + 1] = (R[k * 3 + i] + R[i * 3 + k]) * t;
    }
    if (q[0] < 0) for (double& v : q) v = -v;
    const double sn = std::sqrt(q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    if (sn < 1e-300) { w[0] = 2 * q[1]; w[1] = 2 * q[2]; w[2] = 2 * q[3]; return; }
    const double th = 2.0 * std::atan2(sn, q[0]);
    for (int a = 0; a < 3; ++a) w[a] = q[a + 1] * th / sn;
}
// Eigen AngleAxis(a, Z) * AngleAxis(b, Y) * AngleAxis(c, X)  (Image.h:132-135)
inline void zyx_euler_to_matrix(double a, double b, double c, double R[9]) {
    const double ca = std::cos(a), sa = std::sin(a), cb = std::cos(b), sb = std::sin(b),
                 cc = std::cos(c), sc = std::sin(c);
    R[0] = ca * cb; R[1] = ca * sb * sc - sa * cc; R[2] = ca * sb * cc + sa * sc;
    R[3] = sa * cb; R[4] = sa * sb * sc + ca * cc; R[5] = sa * sb * cc - ca * sc;
    R[6] = -sb;     R[7] = cb * sc;                R[8] = cb * cc;
}
}  // namespace rot

class Camera {
   public:
    using Ptr = std::shared_ptr<Camera>;
    Camera(double fx, double fy, double cx, double cy) : fx(fx), fy(fy), cx(cx), cy(cy) {}
    std::array<double, 4> getIntrinsic() const { return {fx, fy, cx, cy}; }   // Camera.h:94-96
    void setIntrinsic(const std::array<double, 4>& v) { fx = v[0]; fy = v[1]; cx = v[2]; cy = v[3]; }
    double fx, fy, cx, cy;
};

class Image {
   public:
    using Idx = std::size_t;
    using Ptr = std::shared_ptr<Image>;
    explicit Image(Camera::Ptr camera) : idx_(next_idx()), camera_(std::move(camera)) {}
    Idx getIdx() const { return idx_; }
    Camera::Ptr getCamera() const { return camera_; }
    // pose Tcw as angle-axis w (Image.h:88-93) and translation t
    std::array<double, 3> getAngleAxisWc() const { return {pose_[0], pose_[1], pose_[2]}; }
    std::array<double, 3> getTranslation() const { return {pose_[3], pose_[4], pose_[5]}; }
    void setPose(const std::array<double, 6>& p) { pose_ = p; }
    const std::array<double, 6>& pose() const { return pose_; }
    // Reference write-back Image::setIntrinsic(Matx23d) (Image.h:131-141): the
    // three angle-axis numbers are interpreted as ZYX Euler angles.  Kept
    // verbatim in compat mode; `fixed` stores the angle-axis unchanged.
    void setIntrinsic(const std::array<double, 6>& aat, bool fixed = false) {
        if (fixed) { pose_ = aat; return; }
        double R[9], w[3];
        rot::zyx_euler_to_matrix(aat[0], aat[1], aat[2], R);
        rot::matrix_to_aa(R, w);
        pose_ = {w[0], w[1], w[2], aat[3], aat[4], aat[5]};
    }
    // descriptors: n x 128 uint8 (RootSIFT uchar as openMVG regions), keypoints
    std::vector<uint8_t> descriptors;
    std::vector<Point2d> keypoints;
    std::size_t numDescriptors() const { return descriptors.size() / 128; }
    std::unordered_map<std::size_t, std::size_t> kpt_wpt_idx_map_;

   private:
    static Idx next_idx() { static Idx c = 0; return c++; }
    Idx idx_;
    Camera::Ptr camera_;
    std::array<double, 6> pose_{};
};

struct WorldPoint {
    using Ptr = std::shared_ptr<WorldPoint>;
    using Idx = std::size_t;
    Idx idx_ = 0;
    std::array<double, 3> world_pos_{};
    std::vector<uint8_t> last_descriptor_;                               // 128 bytes
    std::vector<std::pair<std::shared_ptr<Image>, Point2d>> observed_frames_;
    void setPos(const std::array<double, 3>& p) { world_pos_ = p; }     // WorldPoint.h:35-40
};

class LocalFrame;
template <class Solver> class BasicBundleAdjuster;

class WorldStructure {
   public:
    using Ptr = std::shared_ptr<WorldStructure>;
    void addImage(const Image::Ptr& img) { images_[img->getIdx()] = img; }
    WorldPoint::Idx addPoint(const std::array<double, 3>& pos, std::vector<uint8_t> descriptor) {
        auto p = std::make_shared<WorldPoint>();
        p->idx_ = cur_idx_++;
        p->world_pos_ = pos;
        p->last_descriptor_ = std::move(descriptor);
        desc_.resize(desc_.size() + 128, 0);
        std::copy_n(p->last_descriptor_.begin(), std::min<std::size_t>(128, p->last_descriptor_.size()),
                    desc_.end() - 128);
        world_points_[p->idx_] = p;
        by_idx_.push_back(p);
        return p->idx_;
    }
    // a point's latest descriptor (WorldPoint::last_descriptor_, kept in step
    // with the index-ordered copy GlobalFrame matches against)
    void setLastDescriptor(WorldPoint::Idx i, std::vector<uint8_t> descriptor) {
        std::copy_n(descriptor.begin(), std::min<std::size_t>(128, descriptor.size()), desc_.begin() + 128 * i);
        by_idx_[i]->last_descriptor_ = std::move(descriptor);
    }
    // a new observation of a point (its observed_frames_ list, and the count)
    void addObservation(const WorldPoint::Ptr& p, std::shared_ptr<Image> im, Point2d uv) {
        p->observed_frames_.emplace_back(std::move(im), uv);
        ++n_obs_;
    }
    int64_t observationCount() const { return n_obs_; }
    void addLocalFrame(std::shared_ptr<LocalFrame> f) { local_frames_.push_back(std::move(f)); }
    const std::vector<std::shared_ptr<LocalFrame>>& getLocalFrames() const { return local_frames_; }
    WorldPoint::Ptr getPointFromIdx(WorldPoint::Idx i) const { return world_points_.at(i); }
    const std::unordered_map<WorldPoint::Idx, WorldPoint::Ptr>& points() const { return world_points_; }
    // the same points in index order (points are only ever added, with
    // increasing indices): what GlobalFrame iterates, without a sort per image
    const std::vector<WorldPoint::Ptr>& pointsByIdx() const { return by_idx_; }
    // every point's last descriptor, 128 bytes each, in index order
    const std::vector<uint8_t>& descriptorsByIdx() const { return desc_; }

   private:
    WorldPoint::Idx cur_idx_ = 0;
    std::vector<std::shared_ptr<LocalFrame>> local_frames_;
    std::unordered_map<Image::Idx, Image::Ptr> images_;
    std::unordered_map<WorldPoint::Idx, WorldPoint::Ptr> world_points_;
    std::vector<WorldPoint::Ptr> by_idx_;
    std::vector<uint8_t> desc_;     // [points][128]
    int64_t n_obs_ = 0;
    template <class> friend class BasicBundleAdjuster;
    friend class GlobalFrame;
};

}  // namespace sfm
