// rtx_collapse.h — the collapsed walk: box tests a threaded walk may leave out (rtx_collapse.hip;
// host code).
//
// A node's box is the union of its children's (NewAabbFromBoxes, bvh.go:44-50: Go's min / max,
// exact in float32), so a child's box lies inside its parent's.  InBoundary (bvh.go:84-102) is
// monotone in the box: (min - o) * invD and (max - o) * invD are monotone in min / max under IEEE
// rounding, and a NaN (0 * inf) only ever loosens the parent's interval.  So a child passes only
// where its parent passes, with the same running bound.  A walk that leaves out a node's box test
// and goes straight to the node's children therefore tests the same primitives, in the same
// order, against the same bounds: every hit, every path and every image bit stays the same; only
// the number of box tests changes — one fewer where the node passes, (children - 1) more where
// it fails.
//
// Which tests to leave out is a cost choice: with P(X) the number of times node X's box passes,
// a kept set K costs sum over X in K of P(nearest kept ancestor of X) box tests.  P is estimated
// on a few thousand host-side sample paths from the camera (plain closest-hit walks with diffuse
// bounces — an estimate only, never an image), and K is the exact optimum for that estimate (a
// dynamic programme over the tree).  A node keeps its test when any child is a primitive (a
// primitive's test must stay behind its own box, since the float32 sphere test can report hits
// outside it) or when a child's box is not inside its own (a caller's hand-made
// table may not nest; NewBVH's always does).
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/rtx.h"
#include "rtx_layout.h"

namespace rtxd {

// How often each node entry of the threaded layout E (rtx_layout.h host form: escapes are entry
// indices) passes its box test on sample paths from camera `cam`; pass[i] = 0 for primitives.
// *walks = the number of walks (each starts at entry 0).  quadtab: 16 floats per quad.
void sample_node_passes(const std::vector<rtx_entry>& E, const std::vector<float>& quadtab, const rtx_camera& cam,
                        std::vector<double>& pass, double* walks);

// The collapsed layout of E for pass estimates `pass` / `walks`: out = E without the node entries
// the optimum leaves out (none unless allow_drop), escapes renumbered.  skip[k] = 1 when the k-th
// node entry of E (in E's order) is left out; reads (optional) = each out entry's estimated reads
// (the passes of its nearest kept ancestor).  Returns false (out = E, no skips, no reads) when the
// tree is too deep to plan.
bool collapse_layout(const std::vector<rtx_entry>& E, const std::vector<double>& pass, double walks, bool allow_drop,
                     std::vector<rtx_entry>& out, std::vector<uint8_t>& skip, std::vector<double>* reads);

}  // namespace rtxd
