// rtx_topology.h — the walk's own tree over a sphere scene (rtx_topology.hip; host code).
//
// The reference's tree (NewBVH, bvh.go:142-185) splits at the median of a random axis, so its
// boxes overlap heavily: 38 box and 6 sphere tests per segment on randSpheres, 97 box tests on
// config 4.  Its closest hit (bvh.go:220-249) is the nearest root among the spheres the ray
// reaches — those whose boxes, all the way down, the ray passes — so another tree over the same
// spheres gives the same answer when every sphere is reachable by the same rays.
//
// GUARDED (the default): the units of the rebuilt tree are the reference tree's leaves, the
// nodes NewBVH makes for one or two spheres (bvh.go:162-174), with their boxes and their spheres
// in their order.  Above them sits a binned surface-area-heuristic tree whose boxes are unions of
// unit boxes.  Every sphere keeps the reference's innermost box as its innermost box and every
// box above it contains that box, so (slab tests being monotone in the box) a ray reaches a
// sphere here exactly when it reaches it in the reference's tree, with the same running bound
// semantics; only the order of the units changes.
// UNGUARDED (RTX_BVH=sah, A/B): the units are the spheres themselves (own boxes).  The reachable
// set can then differ where the float32 sphere test reports hits outside a sphere's box
// (DESIGN.md §12 measures where).
//
// NEAR (the tiered walk): the units are the spheres, each behind its own box grown
// by the float32 sphere test's error bound for ray origins inside a NEAR REGION (near_region):
// a hit the test reports from there lies inside that box, so such rays reach every sphere they
// can hit.  Rays from outside the region walk the guarded tree instead (the kernel's far pass).
//
// Either tree is walked near child first along the camera's viewing direction: one threaded
// layout per camera octant, made on first use.
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/rtx.h"
#include "rtx_layout.h"

namespace rtxd {

struct Topology {
    bool guarded = true;
    bool near = false;     // unguarded units behind boxes grown for origins in near_box
    float near_box[6] = {};  // min xyz, max xyz (near trees)
    uint32_t n_internal = 0;          // SAH nodes: nodes[0 .. n_internal)
    // nodes: the SAH nodes (children in canonical order: left = the low side of the split), then
    // (guarded) one copy of each unit's node with its sphere refs
    std::vector<rtx_bvh_node> nodes;
    std::vector<uint8_t> axis;        // split axis of each SAH node
    std::vector<int32_t> child_unit;  // 2 per SAH node: the unit its left / right child is, or -1
    int32_t root = 0;
    // per unit: its entries in the reference's layout (guarded: the node, then its spheres;
    // unguarded: the sphere), concatenated; unit u = unit_entries[unit_first[u] .. unit_first[u+1])
    std::vector<rtx_entry> unit_entries;
    std::vector<uint32_t> unit_first;
};

// The tree over the spheres of `ref`, the threaded entries emitted from the caller's tree
// (rtx_layout.h, reference order).  Returns false (out untouched) when the tree does not qualify:
// anything but spheres, a sphere outside a leaf node of one or two spheres (guarded), or fewer
// than two units.
// near_box (unguarded only): grow every sphere's box by sphere_margin for origins in that box.
// quadtab (the scene's quad table, rtx_layout.h, 16 floats per quad): a near tree holds the quads too, each behind
// its corners' box grown by quad_margin.
bool build_topology(const std::vector<rtx_entry>& ref, bool guarded, Topology& out, const float* near_box = nullptr,
                    const std::vector<float>* quadtab = nullptr);

// The near region of a tiered walk: the box of the spheres that are not huge (precise_enough's
// core) grown by `grow` times its largest extent on every side, min xyz then max xyz.  False when
// the scene has no finite core.
// quadtab: the quads' own boxes join the core (a scene of quads only: they are the core).
bool near_region(const std::vector<rtx_entry>& ref, float box[6], double grow = 1.0,
                 const std::vector<float>* quadtab = nullptr);

// NewQuad's box, NewAabb(Q, Q + u + v).GetPaddedAabb() (hittables.go:162, bvh.go:63-84), in float32 as Go forms it,
// of the quad record q (16 floats of the quad table).
void quad_own_box(const float* q, float mn[3], float mx[3]);

// How far from its parallelogram the float32 quad test (hittables.go:167-190) can put a hit for a ray origin whose
// coordinates are within omax, with room for the slab test's rounding: K u (|u| + |v| + 2B + 3 omax)(2 + 2 / sin)
// + 4u (B + omax), B bounding the quad's coordinates, sin the sine of the angle of u and v, K = 64 (RTX_MARGIN_KQ
// widens it).  DESIGN.md §26 derives the terms; tests/test_tier.py meets at most a small fraction of it.
double quad_margin(const float* q, double omax);

// How far outside a sphere (centre c, radius r) the float32 sphere test (hittables.go:96-116) can
// put a hit for a ray origin at distance <= dmax from c (its coordinates <= omax in magnitude), with
// room for the slab test's rounding in either form (the reference's and the near walk's FMA form):
// rho - r + 2^-20 (dmax + rho) + 2^-23 omax, rho = sqrt(r^2 + 24u (dmax^2 + r^2)), u = 2^-24 — the
// forward-error bound derived in DESIGN.md §15.1 (the computed discriminant is within
// 24u |d|^2 (D^2 + r^2) of the exact one; the adversarial test meets at most 8.1u).
double sphere_margin(double r, double dmax, double omax);

// Whether the scene's spheres are small against the float32 sphere test's error (see the .hip):
// the gate of the default (guarded) rebuild.
bool precise_enough(const std::vector<rtx_entry>& ref);

// Whether every node box of the caller's walk `ref` contains the own box (NewSphere's NewAabb,
// hittables.go:85-94) of every sphere below it, and the scene holds spheres only: the tiered walk's
// hit check accepts a near-tree hit by testing the sphere's own box in place of every
// box the far walk would test above it.  NewBVH's nodes always qualify (NewAabbFromBoxes, bvh.go:44-50).
// quadtab: the scene's quads too, each with its own box (quad_own_box).
bool own_boxes_nested(const std::vector<rtx_entry>& ref, const std::vector<float>* quadtab = nullptr);

// The node table of `t` as walked for camera octant `oct` (bit k: the viewing direction is
// negative along axis k): at every SAH node the child on the near side of its split along the
// viewing direction is `left`, the one visited first.  Unit nodes keep the reference's order.
void orient_topology(const Topology& t, uint32_t oct, std::vector<rtx_bvh_node>& out);

// The threaded entries (rtx_layout.h) of `t` walked for octant `oct`.
void emit_topology(const Topology& t, uint32_t oct, std::vector<rtx_entry>& out);

// Octant of a camera's viewing direction (pixel00 + du W/2 + dv H/2 - center).
uint32_t camera_octant(const rtx_camera& c);

}  // namespace rtxd
