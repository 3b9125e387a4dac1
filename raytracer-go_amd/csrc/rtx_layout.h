// rtx_layout.h — device layout of a scene (library-internal; not part of the ABI).
//
// The reference walks a pointer tree recursively on every ray (bvh.go:220-249):
// box test, left child, right child clipped to the left hit.  That visit order is a
// pre-order depth-first walk with a running "closest" bound.  On the device the tree
// is stored as that walk, "threaded": one 32-B entry per node / primitive in
// pre-order, and every node carries its escape index (the entry after its subtree).
//
//   node box hit  -> next = i + 1          (descend: first child in pre-order)
//   node box miss -> next = escape         (skip the subtree)
//   primitive     -> test, next = i + 1
//
// So traversal needs no stack at all and visits exactly the reference's sequence
// of box and primitive tests with the same running bound — the results are
// bit-identical to the recursion, including ties (left before right).  The one
// deliberate difference: a one-element split stores left == right (bvh.go:162-165);
// its second test can never succeed (open interval clipped to the first hit, or an
// identical miss), so that primitive is emitted once.
//
// Entry (two float4 = 32 B, 16-B aligned; loads are 2 x global/ds 128-bit):
//   node:   a = (bmin.x, bmin.y, bmin.z, int escape)   b = (bmax.x, bmax.y, bmax.z, int RTX_E_NODE)
//   sphere: a = (c.x, c.y, c.z, radius)                b = (radius*radius, int sphere, 0, int material >= 0)
//   quad:   a = (normal.x, normal.y, normal.z, D)      b = (int quad, 0, 0, int RTX_E_QUAD)
// A quad's plane test needs only its entry; the in-plane test and shading read its
// record from the quad table that follows the entries (4 float4 per quad):
//   (Q.x, Q.y, Q.z, int material), (u, 0), (v, 0), (w, 0)   — NewQuad's fields,
// hittables.go:149-165, computed on the host.
// radius*radius is the float32 product hittables.go:100 computes, precomputed.
// On the device the halves live in two arrays (all a, then all b: rtxd::SceneRef), so
// a wave's gathers spread over every LDS bank group, and the integer words are recoded
// so that a step needs no index arithmetic (rtx_capi.hip, ensure_device):
//   positions are byte offsets, 16 * index (rtxd::Trav::i);
//   node:   a.w = escape position, b.w = next position  (b.w >= 0 <=> node)
//   sphere: b.z = next position, b.w = RTX_DEV_SPHERE(material) = -3 - material
//   quad:   b.z = next position, b.w = RTX_E_QUAD
// Since every entry names its successor, the storage order is free: it is the walk order,
// except that a scene too big for the LDS copy stores its top levels first (v3 caches those
// in LDS; ensure_device).  The walk order, and so every test and its result, is unchanged.
// Each array ends with one extra entry, the sentinel at index n: a node with an empty
// box whose escape and next are both its own position.  Every walk ends there and a
// step on it changes nothing, whatever the ray (NaN included), so lanes that are not
// traversing take the same steps as those that are (rtxd::traverse_phase) instead of
// being masked off one step at a time.
#pragma once
#include <stdint.h>

#define RTX_E_NODE (-1)
#define RTX_E_QUAD (-2)
#define RTX_DEV_SPHERE(material) (-3 - (int32_t)(material))
#define RTX_DEV_SPHERE_MATERIAL(tag) ((uint32_t)(-3 - (tag)))

struct rtx_entry {
    float a[4];
    float b[4];
};
static_assert(sizeof(rtx_entry) == 32, "entry is 32 B");
