// bvh.cpp — internal/bvh.go: Interval, Aabb and the BVH build (host, once per scene).
// The hot half of bvh.go (Aabb.Hit / BVH.Hit, :52-61, :84-102, :220-249) runs on
// the device (csrc/rtx_device.h, closest_hit).
#include <algorithm>

#include "internal.h"

namespace internal {

Interval NewInterval(float min, float max) { return Interval{min, max}; }

Aabb NewAabb(const Vec3& p1, const Vec3& p2) {  // bvh.go:28-34
    return Aabb{NewInterval(MinF32(p1.X, p2.X), MaxF32(p1.X, p2.X)), NewInterval(MinF32(p1.Y, p2.Y), MaxF32(p1.Y, p2.Y)),
                NewInterval(MinF32(p1.Z, p2.Z), MaxF32(p1.Z, p2.Z))};
}

Aabb NewAabbFromIntervals(Interval x, Interval y, Interval z) { return Aabb{x, y, z}; }  // bvh.go:36-42

Aabb NewAabbFromBoxes(const Aabb& b1, const Aabb& b2) {  // bvh.go:44-50
    return Aabb{NewInterval(MinF32(b1.x.min, b2.x.min), MaxF32(b1.x.max, b2.x.max)),
                NewInterval(MinF32(b1.y.min, b2.y.min), MaxF32(b1.y.max, b2.y.max)),
                NewInterval(MinF32(b1.z.min, b2.z.min), MaxF32(b1.z.max, b2.z.max))};
}

Aabb Aabb::GetPaddedAabb() const {  // bvh.go:63-82
    const float eps = 0.0001f;
    Interval px = x, py = y, pz = z;
    if (px.max - px.min < eps) { px.min -= eps; px.max += eps; }
    if (py.max - py.min < eps) { py.min -= eps; py.max += eps; }
    if (pz.max - pz.min < eps) { pz.min -= eps; pz.max += eps; }
    return NewAabbFromIntervals(px, py, pz);
}

std::shared_ptr<BVH> NewBVHFromWorld(const World& w) { return NewBVH(w.hittables); }  // bvh.go:138-140

// HittableCompare{X,Y,Z}, bvh.go:187-218: +1 when h2's min is larger (=> descending).
static int compare_axis(const HittablePtr& h1, const HittablePtr& h2, int axis) {
    const Aabb b1 = h1->GetBounds(), b2 = h2->GetBounds();
    const float m1 = axis == 0 ? b1.x.min : (axis == 1 ? b1.y.min : b1.z.min);
    const float m2 = axis == 0 ? b2.x.min : (axis == 1 ? b2.y.min : b2.z.min);
    const float diff = m2 - m1;
    if (diff > 0) return 1;
    if (diff < 0) return -1;
    return 0;
}

// NewBVH, bvh.go:142-185.  The axis comes from the global source (rand.Intn(3), drawn
// before the size switch, so also for 1- and 2-element lists).  The sort is stable:
// x/exp/slices.SortFunc is an unstable pdqsort, so equal keys may land in either
// order in the reference — the contract fixes one of its possible outcomes.
std::shared_ptr<BVH> NewBVH(const std::vector<HittablePtr>& hittables) {
    auto bvh = std::make_shared<BVH>();
    std::vector<HittablePtr> h(hittables);  // :144-145
    const int axis = GlobalRand().Intn(3);  // :147
    switch (h.size()) {
    case 0:
        return nullptr;  // the reference indexes h[0] here; the mirror refuses
    case 1:  // :162-165
        bvh->left = h[0];
        bvh->right = h[0];
        break;
    case 2:  // :166-174
        if (compare_axis(h[0], h[1], axis) > 0) {
            bvh->left = h[1];
            bvh->right = h[0];
        } else {
            bvh->left = h[0];
            bvh->right = h[1];
        }
        break;
    default: {  // :175-180
        std::stable_sort(h.begin(), h.end(),
                         [axis](const HittablePtr& a, const HittablePtr& b) { return compare_axis(a, b, axis) < 0; });
        const size_t mid = h.size() / 2;
        bvh->left = NewBVH(std::vector<HittablePtr>(h.begin(), h.begin() + (long)mid));
        bvh->right = NewBVH(std::vector<HittablePtr>(h.begin() + (long)mid, h.end()));
    }
    }
    bvh->bBox = NewAabbFromBoxes(bvh->left->GetBounds(), bvh->right->GetBounds());  // :182
    return bvh;
}

}  // namespace internal
