// LocalFrame / GlobalFrame (src/frame/LocalFrame.h:19-83, GlobalFrame.h:15-79)
// over any matcher with the cv::DescriptorMatcher::knnMatch(query, train,
// out, k = 1) shape.  The product binds them to sfm::Matcher (GPU, sfm.hpp);
// the loop oracle binds them to the CPU restatement.  Header-only, no
// dependency on the C-ABI.
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstring>
#include <memory>
#include <vector>

#include "world.hpp"

namespace sfm {

class LocalFrame {
   public:
    using Ptr = std::shared_ptr<LocalFrame>;
    LocalFrame(Image::Ptr image1, Image::Ptr image2) : image1_(std::move(image1)), image2_(std::move(image2)) {}
    Image::Ptr getImage1() const { return image1_; }
    Image::Ptr getImage2() const { return image2_; }
    const std::vector<DMatch>& getMatches() const { return matches_; }
    // knnMatch(image1 descriptors, image2 descriptors, k = 1); rows without a
    // (cross-checked) partner are skipped (LocalFrame.h:31-47)
    template <class M> std::size_t matchFeature(M& matcher) {
        if (!matches_.empty()) matches_.clear();  // "Rematch feature" warning in the reference
        std::vector<std::vector<DMatch>> v;
        matcher.knnMatch(image1_->descriptors, image2_->descriptors, v, 1);
        for (auto& row : v)
            if (!row.empty()) matches_.push_back(row[0]);
        raw_ = matches_.size();
        return matches_.size();
    }
    std::size_t rawMatchCount() const { return raw_; }   // before the filter
    // keep d <= 4 * min d (LocalFrame.h:49-64); empty input -> empty (the
    // reference dereferences min_element of an empty vector)
    std::vector<DMatch> filterMatches() const {
        std::vector<DMatch> good;
        if (matches_.empty()) return good;
        const float mn = std::min_element(matches_.begin(), matches_.end(),
                                          [](const DMatch& a, const DMatch& b) { return a.distance < b.distance; })
                             ->distance;
        for (const auto& m : matches_)
            if (m.distance <= 4 * mn) good.push_back(m);
        return good;
    }
    template <class M> std::size_t matchFeatureAndFilter(M& matcher) {  // :66-70
        matchFeature(matcher);
        matches_ = filterMatches();
        return matches_.size();
    }

   private:
    Image::Ptr image1_, image2_;
    std::vector<DMatch> matches_;
    std::size_t raw_ = 0;
};

class GlobalFrame {
   public:
    // world points in index order (the reference iterates its unordered_map,
    // GlobalFrame.h:16-20; index order is the deterministic choice)
    // (the world outlives the frame: it keeps the world's index-ordered list)
    GlobalFrame(const WorldStructure::Ptr& world, Image::Ptr image)
        : image_(std::move(image)), world_points_(&world->pointsByIdx()), world_desc_(&world->descriptorsByIdx()) {}
    // query = every world point's last_descriptor_ (the world keeps them in
    // one index-ordered array), train = the image (:22-43)
    template <class M> std::size_t matchFeature(M& matcher) {
        matches_.clear();
        std::vector<std::vector<DMatch>> v;
        matcher.knnMatch(*world_desc_, image_->descriptors, v, 1);
        for (auto& row : v)
            if (!row.empty()) matches_.push_back(row[0]);
        raw_ = matches_.size();
        return matches_.size();
    }
    std::size_t rawMatchCount() const { return raw_; }   // before the filter
    // drop d > 3 * min d (GlobalFrame.h:45-60)
    std::vector<DMatch> filterMatches() const {
        std::vector<DMatch> good;
        if (matches_.empty()) return good;
        float mn = matches_[0].distance;
        for (auto& m : matches_) mn = std::min(mn, m.distance);
        for (auto& m : matches_)
            if (!(m.distance > 3 * mn)) good.push_back(m);
        return good;
    }
    template <class M> std::size_t matchFeatureAndFilter(M& matcher) {  // :62-66
        matchFeature(matcher);
        matches_ = filterMatches();
        return matches_.size();
    }
    const std::vector<WorldPoint::Ptr>& get_world_points() const { return *world_points_; }
    const std::vector<DMatch>& getMatches() const { return matches_; }

   private:
    std::vector<DMatch> matches_;
    Image::Ptr image_;
    const std::vector<WorldPoint::Ptr>* world_points_;
    const std::vector<uint8_t>* world_desc_;
    std::size_t raw_ = 0;
};

}  // namespace sfm
