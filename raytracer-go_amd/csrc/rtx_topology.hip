// rtx_topology.hip — the walk's own tree over a sphere scene, and the near tree of a tiered walk (host code; see
// rtx_topology.h).
#include "rtx_topology.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace rtxd {
namespace {

// Go's math.Min / math.Max on float32 operands (bvh.go:28-50 via math.go:38-44): NaN wins,
// -0 below +0.
float go_min(float a, float b) {
    if (a != a || b != b) return NAN;
    if (a == 0.0f && b == 0.0f) return std::signbit(a) ? a : b;
    return a < b ? a : b;
}
float go_max(float a, float b) {
    if (a != a || b != b) return NAN;
    if (a == 0.0f && b == 0.0f) return std::signbit(a) ? b : a;
    return a > b ? a : b;
}

struct Box {
    float mn[3], mx[3];
};

Box unite(const Box& a, const Box& b) {  // NewAabbFromBoxes, bvh.go:44-50
    Box r;
    for (int k = 0; k < 3; ++k) {
        r.mn[k] = go_min(a.mn[k], b.mn[k]);
        r.mx[k] = go_max(a.mx[k], b.mx[k]);
    }
    return r;
}

double half_area(const double lo[3], const double hi[3]) {
    const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return dx * dy + dy * dz + dz * dx;
}

int32_t tag_of(const rtx_entry& e) {
    int32_t t;
    std::memcpy(&t, &e.b[3], 4);
    return t;
}
int32_t word(const float* f) {
    int32_t t;
    std::memcpy(&t, f, 4);
    return t;
}

// Binned-SAH tree over `boxes` (one leaf per item): appends the SAH nodes to out.nodes /
// out.axis / out.child_unit, item j becoming child ref item_ref[j].
void build_sah(const std::vector<Box>& boxes, const std::vector<int32_t>& item_ref, Topology& out,
               std::vector<int32_t>& child_unit) {
    const uint32_t n = (uint32_t)boxes.size();
    std::vector<uint32_t> ids(n);
    for (uint32_t i = 0; i < n; ++i) ids[i] = i;
    std::vector<double> cen(3 * (size_t)n);  // box centres (binning only)
    for (uint32_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) cen[3 * i + k] = 0.5 * ((double)boxes[i].mn[k] + (double)boxes[i].mx[k]);
    struct Task {
        int32_t node;
        uint32_t first, count;
    };
    std::vector<Task> stack;
    auto new_node = [&]() {
        out.nodes.push_back(rtx_bvh_node{});
        out.axis.push_back(0);
        child_unit.push_back(-1);
        child_unit.push_back(-1);
        return (int32_t)(out.nodes.size() - 1);
    };
    out.root = new_node();
    stack.push_back({out.root, 0, n});
    constexpr int NB = 32;
    auto bin_of = [](double c, double lo, double ext) {  // NaN centres go to bin 0
        const double v = (c - lo) * (NB / ext);
        return v >= 0.0 ? (v < NB ? (int)v : NB - 1) : 0;
    };
    while (!stack.empty()) {
        const Task t = stack.back();
        stack.pop_back();
        uint32_t* I = ids.data() + t.first;
        Box b = boxes[I[0]];
        double clo[3], chi[3];
        for (int k = 0; k < 3; ++k) clo[k] = chi[k] = cen[3 * I[0] + k];
        for (uint32_t i = 1; i < t.count; ++i) {
            b = unite(b, boxes[I[i]]);
            for (int k = 0; k < 3; ++k) {
                clo[k] = std::min(clo[k], cen[3 * I[i] + k]);
                chi[k] = std::max(chi[k], cen[3 * I[i] + k]);
            }
        }
        std::memcpy(out.nodes[t.node].bmin, b.mn, sizeof(b.mn));
        std::memcpy(out.nodes[t.node].bmax, b.mx, sizeof(b.mx));
        // cost of a split: A(left) N(left) + A(right) N(right), over NB centre bins per axis
        double best = INFINITY;
        int bax = -1, bsplit = -1;
        for (int ax = 0; ax < 3; ++ax) {
            const double ext = chi[ax] - clo[ax];
            if (!(ext > 0.0) || !std::isfinite(ext)) continue;
            double blo[NB][3], bhi[NB][3];
            uint32_t bc[NB] = {0};
            for (int q = 0; q < NB; ++q)
                for (int k = 0; k < 3; ++k) {
                    blo[q][k] = INFINITY;
                    bhi[q][k] = -INFINITY;
                }
            for (uint32_t i = 0; i < t.count; ++i) {
                const int q = bin_of(cen[3 * I[i] + ax], clo[ax], ext);
                ++bc[q];
                for (int k = 0; k < 3; ++k) {
                    blo[q][k] = std::min(blo[q][k], (double)boxes[I[i]].mn[k]);
                    bhi[q][k] = std::max(bhi[q][k], (double)boxes[I[i]].mx[k]);
                }
            }
            double ra[NB], lo[3], hi[3];
            uint32_t rc[NB], cnt = 0;
            for (int k = 0; k < 3; ++k) {
                lo[k] = INFINITY;
                hi[k] = -INFINITY;
            }
            for (int q = NB - 1; q > 0; --q) {
                for (int k = 0; k < 3; ++k) {
                    lo[k] = std::min(lo[k], blo[q][k]);
                    hi[k] = std::max(hi[k], bhi[q][k]);
                }
                cnt += bc[q];
                ra[q] = cnt ? half_area(lo, hi) : 0.0;
                rc[q] = cnt;
            }
            for (int k = 0; k < 3; ++k) {
                lo[k] = INFINITY;
                hi[k] = -INFINITY;
            }
            cnt = 0;
            for (int q = 0; q < NB - 1; ++q) {
                for (int k = 0; k < 3; ++k) {
                    lo[k] = std::min(lo[k], blo[q][k]);
                    hi[k] = std::max(hi[k], bhi[q][k]);
                }
                cnt += bc[q];
                if (cnt == 0 || rc[q + 1] == 0) continue;
                const double c = half_area(lo, hi) * cnt + ra[q + 1] * rc[q + 1];
                if (c < best) {
                    best = c;
                    bax = ax;
                    bsplit = q;
                }
            }
        }
        uint32_t mid = t.count / 2;  // every centre equal (or not finite): split the list in the middle
        if (bax >= 0) {
            const double ext = chi[bax] - clo[bax];
            auto low = [&](uint32_t id) { return bin_of(cen[3 * id + bax], clo[bax], ext) <= bsplit; };
            mid = (uint32_t)(std::stable_partition(I, I + t.count, low) - I);
            if (mid == 0 || mid == t.count) mid = t.count / 2;
        } else {
            bax = 0;
        }
        out.axis[t.node] = (uint8_t)bax;
        const uint32_t cnt[2] = {mid, t.count - mid}, first[2] = {t.first, t.first + mid};
        int32_t child[2];
        for (int c = 0; c < 2; ++c) {
            if (cnt[c] == 1) {
                child[c] = item_ref[ids[first[c]]];
                child_unit[2 * t.node + c] = (int32_t)ids[first[c]];
            } else {
                child[c] = new_node();
                stack.push_back({child[c], first[c], cnt[c]});
            }
        }
        out.nodes[t.node].left = child[0];
        out.nodes[t.node].right = child[1];
    }
}

}  // namespace

void quad_own_box(const float* q, float mn[3], float mx[3]) {
    // NewAabb(Q, Q + u + v).GetPaddedAabb() (hittables.go:162, bvh.go:28-34, 63-84): Add(Add(Q, u), v) in float32,
    // Go's Min / Max, then every axis thinner than 0.0001 widened by 0.0001 on both sides (float32 operations)
    const float eps = 0.0001f;
    for (int k = 0; k < 3; ++k) {
        volatile float c = q[k] + q[4 + k];  // (no contraction: the reference's two float32 additions)
        c = c + q[8 + k];
        const float p1 = q[k], p2 = c;
        float lo = go_min(p1, p2), hi = go_max(p1, p2);
        volatile float ext = hi - lo;
        if (ext < eps) {
            lo = lo - eps;
            hi = hi + eps;
        }
        mn[k] = lo;
        mx[k] = hi;
    }
}

// RTX_MARGIN_KQ (read once; default 64, at least 64): the constant K of quad_margin's bound.
static double margin_kq() {
    static const double k = [] {
        const char* e = std::getenv("RTX_MARGIN_KQ");
        const double v = e ? std::strtod(e, nullptr) : 64.0;
        return v >= 64.0 && std::isfinite(v) ? v : 64.0;
    }();
    return k;
}

double quad_margin(const float* q, double omax) {
    const double u[3] = {q[4], q[5], q[6]}, v[3] = {q[8], q[9], q[10]};
    const double n[3] = {u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0]};
    const double U = std::sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]), V = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    const double S = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    if (!(S > 0.0) || !std::isfinite(S) || !(U > 0.0) || !(V > 0.0)) return INFINITY;  // degenerate: no near box
    double B = 0.0;  // a bound on the coordinates of points of the quad
    for (int k = 0; k < 3; ++k) B = std::max(B, std::fabs((double)q[k]) + std::fabs(u[k]) + std::fabs(v[k]));
    const double sin_t = S / (U * V);
    const double m = std::ldexp(margin_kq() * (U + V + 2.0 * B + 3.0 * omax) * (2.0 + 2.0 / sin_t), -24);
    return m + std::ldexp(B + omax + m, -21);  // + 4u (|b| + |o|): the slab test's rounding, either form
}

namespace {
// The box of the spheres that are not huge (a sphere is huge when its radius exceeds the extent
// of all smaller ones: main.go's ground, r = 1000), and the smallest radius.
bool core_box(const std::vector<rtx_entry>& ref, Box& core, double& rmin, const std::vector<float>* quadtab = nullptr) {
    std::vector<std::pair<float, uint32_t>> rad;  // (radius, entry), spheres only
    for (uint32_t i = 0; i < ref.size(); ++i)
        if (tag_of(ref[i]) >= 0) rad.push_back({std::fabs(ref[i].a[3]), i});
    // quads (the near region of a scene with quads): their own boxes join the core, which they hold when the
    // scene has no sphere
    bool have_q = false;
    Box qb;
    for (uint32_t i = 0; quadtab && i < ref.size(); ++i)
        if (tag_of(ref[i]) == RTX_E_QUAD) {
            Box b;
            quad_own_box(&(*quadtab)[16 * (size_t)word(&ref[i].b[0])], b.mn, b.mx);
            qb = have_q ? unite(qb, b) : b;
            have_q = true;
        }
    if (rad.empty()) {
        if (!have_q) return false;
        core = qb;
        rmin = 0.0;
        return true;
    }
    std::sort(rad.begin(), rad.end());
    std::vector<Box> pre(rad.size());  // union of the boxes of the k + 1 smallest spheres
    for (size_t k = 0; k < rad.size(); ++k) {
        const rtx_entry& e = ref[rad[k].second];
        Box b;
        for (int q = 0; q < 3; ++q) {
            b.mn[q] = e.a[q] - rad[k].first;
            b.mx[q] = e.a[q] + rad[k].first;
        }
        pre[k] = k ? unite(pre[k - 1], b) : b;
    }
    size_t keep = rad.size();  // drop the huge spheres, largest first
    while (keep > 1) {
        const Box& b = pre[keep - 2];
        const double ext = std::max({(double)b.mx[0] - b.mn[0], (double)b.mx[1] - b.mn[1], (double)b.mx[2] - b.mn[2]});
        if (!(rad[keep - 1].first > ext)) break;
        --keep;
    }
    core = have_q ? unite(pre[keep - 1], qb) : pre[keep - 1];
    rmin = rad[0].first;
    return true;
}
}  // namespace

// The float32 sphere test (hittables.go:96-116) forms c = |oc|^2 - r^2 from squares of order D^2
// (D: the ray origin's distance to the centre), so it reports hits up to about eps D^2 / r outside a
// sphere's silhouette.  Where such hits can reach past the innermost box, the order in which two
// units are tried can decide which of two nearby spheres is the closest hit, so the
// tree is rebuilt only where that zone is a small fraction of the spheres: eps D^2 / r_min^2 < 2^-7,
// D the diagonal of the scene without its huge spheres (a sphere is huge when its radius exceeds the
// extent of all smaller ones: main.go's ground, r = 1000).  randSpheres and the config-5 scene pass
// (1.4e-3); config 4's 316-unit slab of r = 0.2 spheres fails (0.3).
bool precise_enough(const std::vector<rtx_entry>& ref) {
    Box b;
    double rmin = 0.0;
    if (!core_box(ref, b, rmin)) return false;
    double d2 = 0.0;
    for (int q = 0; q < 3; ++q) d2 += ((double)b.mx[q] - b.mn[q]) * ((double)b.mx[q] - b.mn[q]);
    return rmin > 0.0 && std::ldexp(d2, -24) / (rmin * rmin) < std::ldexp(1.0, -7);
}

bool own_boxes_nested(const std::vector<rtx_entry>& ref, const std::vector<float>* quadtab) {
    std::vector<uint32_t> open;  // the nodes whose subtree holds entry i (host layout: a[3] = escape index)
    bool any = false;
    for (uint32_t i = 0; i < ref.size(); ++i) {
        while (!open.empty() && (uint32_t)word(&ref[open.back()].a[3]) <= i) open.pop_back();
        const int32_t tag = tag_of(ref[i]);
        if (tag == RTX_E_NODE) {
            open.push_back(i);
            continue;
        }
        if (tag < 0 && !(tag == RTX_E_QUAD && quadtab)) return false;  // a quad (without its table)
        any = true;
        const rtx_entry& e = ref[i];
        float qmn[3], qmx[3];
        if (tag < 0) quad_own_box(&(*quadtab)[16 * (size_t)word(&e.b[0])], qmn, qmx);
        for (int k = 0; k < 3; ++k) {
            const float p1 = e.a[k] + (e.a[3] * -1.0f), p2 = e.a[k] + e.a[3];
            const float mn = tag < 0 ? qmn[k] : go_min(p1, p2), mx = tag < 0 ? qmx[k] : go_max(p1, p2);
            if (!(mn == mn) || !(mx == mx)) return false;
            for (uint32_t n : open)
                if (!(ref[n].a[k] <= mn && ref[n].b[k] >= mx)) return false;
        }
    }
    return any;
}

bool near_region(const std::vector<rtx_entry>& ref, float box[6], double grow, const std::vector<float>* quadtab) {
    Box b;
    double rmin = 0.0;
    if (!core_box(ref, b, rmin, quadtab)) return false;
    double ext = 0.0;
    for (int q = 0; q < 3; ++q) ext = std::max(ext, (double)b.mx[q] - (double)b.mn[q]);
    if (!std::isfinite(ext)) return false;
    for (int q = 0; q < 3; ++q) {  // rounded outward: the region only grows
        box[q] = std::nextafter((float)((double)b.mn[q] - grow * ext), -INFINITY);
        box[3 + q] = std::nextafter((float)((double)b.mx[q] + grow * ext), INFINITY);
        if (!std::isfinite(box[q]) || !std::isfinite(box[3 + q])) return false;
    }
    return true;
}

// The forward-error bound of DESIGN.md §15.1 (u = 2^-24): a computed disc >= 0 puts the ray's line
// within rho = sqrt(r^2 + 24u (D^2 + r^2)) of the centre, and the reported root's point within
// rho + 11u D + 7u rho of it; the slab test of the grown box passes it with 3u (D + r + m) to spare,
// and its FMA form (fma(b, 1/d, -(o/d)), the near walk's: §15.5) with 2u (D + r + m) + u omax, omax
// bounding the origin's coordinates.
// RTX_MARGIN_K (read once; default 24, the derived constant; at least 24) widens the bound's K u (D^2 + r^2) for
// A/B and as a safety factor a caller may want on scenes far from the tested ones (tests/test_tier.py measures
// K <= 8.3 on every adversarial set).
static double margin_k() {
    static const double k = [] {
        const char* e = std::getenv("RTX_MARGIN_K");
        const double v = e ? std::strtod(e, nullptr) : 24.0;
        return v >= 24.0 && std::isfinite(v) ? v : 24.0;
    }();
    return k;
}

double sphere_margin(double r, double dmax, double omax) {
    const double rho = std::sqrt(r * r + std::ldexp(margin_k() * (dmax * dmax + r * r), -24));  // K u, u = 2^-24
    return rho - r + std::ldexp(dmax + rho, -20) + std::ldexp(omax, -23);                       // + 16u (D + rho) + 2u omax
}

bool build_topology(const std::vector<rtx_entry>& ref, bool guarded, Topology& out, const float* near_box,
                    const std::vector<float>* quadtab) {
    if (guarded && near_box) return false;
    // the units, in the reference's walk order: [first entry, end) of each
    std::vector<std::pair<uint32_t, uint32_t>> units;
    const uint32_t n = (uint32_t)ref.size();
    for (uint32_t i = 0; i < n;) {
        const int32_t tag = tag_of(ref[i]);
        if (tag == RTX_E_NODE) {
            const uint32_t e = (uint32_t)word(&ref[i].a[3]);  // escape (host layout: an entry index)
            bool leaf = guarded && e > i + 1 && e <= i + 3 && e <= n;
            for (uint32_t k = i + 1; leaf && k < e; ++k) leaf = tag_of(ref[k]) >= 0;
            if (leaf) {
                units.push_back({i, e});
                i = e;
            } else {
                ++i;
            }
        } else if (tag >= 0 && !guarded) {  // a sphere
            units.push_back({i, i + 1});
            ++i;
        } else if (tag == RTX_E_QUAD && near_box && quadtab) {  // a quad of a near tree
            units.push_back({i, i + 1});
            ++i;
        } else {
            return false;  // a quad, or (guarded) a sphere outside a leaf node
        }
    }
    if (units.size() < 2) return false;
    Topology t;
    t.guarded = guarded;
    if (near_box) {
        t.near = true;
        std::memcpy(t.near_box, near_box, sizeof(t.near_box));
    }
    const uint32_t U = (uint32_t)units.size();
    t.n_internal = U - 1;
    std::vector<Box> boxes(U);
    std::vector<int32_t> item_ref(U);
    t.unit_first.push_back(0);
    for (uint32_t u = 0; u < U; ++u) {
        const rtx_entry& h = ref[units[u].first];
        for (uint32_t k = units[u].first; k < units[u].second; ++k) t.unit_entries.push_back(ref[k]);
        t.unit_first.push_back((uint32_t)t.unit_entries.size());
        if (guarded) {  // the leaf node's own box
            for (int k = 0; k < 3; ++k) {
                boxes[u].mn[k] = h.a[k];
                boxes[u].mx[k] = h.b[k];
            }
            item_ref[u] = (int32_t)(t.n_internal + u);
        } else if (near_box && tag_of(h) == RTX_E_QUAD) {  // the quad's corners' box grown by quad_margin
            const int32_t qi = word(&h.b[0]);
            const float* q = &(*quadtab)[16 * (size_t)qi];
            double omax = 0.0;
            for (int k = 0; k < 6; ++k) omax = std::max(omax, std::fabs((double)near_box[k]));
            const double m = quad_margin(q, omax);
            for (int k = 0; k < 3; ++k) {
                const double c0 = q[k], c1 = c0 + q[4 + k], c2 = c0 + q[8 + k], c3 = c1 + q[8 + k];
                const double lo = std::min({c0, c1, c2, c3}) - m, hi = std::max({c0, c1, c2, c3}) + m;
                boxes[u].mn[k] = std::nextafter((float)lo, -INFINITY);  // rounded outward
                boxes[u].mx[k] = std::nextafter((float)hi, INFINITY);
                if (!(std::fabs(boxes[u].mn[k]) <= 0x1p32f) || !(std::fabs(boxes[u].mx[k]) <= 0x1p32f)) return false;
            }
            item_ref[u] = RTX_REF_PRIM(RTX_PRIM_QUAD, qi);
        } else if (near_box) {  // the sphere's box grown by its margin for origins in the near region
            const double r = std::fabs((double)h.a[3]);
            double d2 = 0.0, omax = 0.0;  // farthest corner of the region from the centre; its largest coordinate
            for (int k = 0; k < 3; ++k) {
                const double lo = (double)near_box[k] - h.a[k], hi = (double)near_box[3 + k] - h.a[k];
                d2 += std::max(lo * lo, hi * hi);
                omax = std::max({omax, std::fabs((double)near_box[k]), std::fabs((double)near_box[3 + k])});
            }
            const double m = sphere_margin(r, std::sqrt(d2), omax);
            for (int k = 0; k < 3; ++k) {  // rounded outward
                boxes[u].mn[k] = std::nextafter((float)((double)h.a[k] - r - m), -INFINITY);
                boxes[u].mx[k] = std::nextafter((float)((double)h.a[k] + r + m), INFINITY);
                // finite, and within 2^32: the near walk's FMA slab form cannot overflow (§15.5)
                if (!(std::fabs(boxes[u].mn[k]) <= 0x1p32f) || !(std::fabs(boxes[u].mx[k]) <= 0x1p32f)) return false;
            }
            item_ref[u] = RTX_REF_PRIM(RTX_PRIM_SPHERE, word(&h.b[1]));
        } else {  // the sphere's box: NewSphere's NewAabb(center - r, center + r), hittables.go:85-94
            for (int k = 0; k < 3; ++k) {
                const float p1 = h.a[k] + (h.a[3] * -1.0f), p2 = h.a[k] + h.a[3];
                boxes[u].mn[k] = go_min(p1, p2);
                boxes[u].mx[k] = go_max(p1, p2);
            }
            item_ref[u] = RTX_REF_PRIM(RTX_PRIM_SPHERE, word(&h.b[1]));
        }
    }
    std::vector<int32_t> child_unit;
    build_sah(boxes, item_ref, t, child_unit);
    if (t.nodes.size() != t.n_internal) return false;  // (a binary tree over U leaves has U - 1 nodes)
    if (guarded) {  // the units' nodes, as the reference built them
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t f = t.unit_first[u], e = t.unit_first[u + 1];
            const rtx_entry& h = t.unit_entries[f];
            rtx_bvh_node nd{};
            for (int k = 0; k < 3; ++k) {
                nd.bmin[k] = h.a[k];
                nd.bmax[k] = h.b[k];
            }
            nd.left = RTX_REF_PRIM(RTX_PRIM_SPHERE, word(&t.unit_entries[f + 1].b[1]));
            nd.right = e - f == 3 ? RTX_REF_PRIM(RTX_PRIM_SPHERE, word(&t.unit_entries[f + 2].b[1])) : nd.left;
            t.nodes.push_back(nd);
        }
    }
    t.child_unit = std::move(child_unit);
    out = std::move(t);
    return true;
}

void orient_topology(const Topology& t, uint32_t oct, std::vector<rtx_bvh_node>& out) {
    out = t.nodes;
    for (uint32_t i = 0; i < t.n_internal; ++i)
        if ((oct >> t.axis[i]) & 1u) std::swap(out[i].left, out[i].right);
}

void emit_topology(const Topology& t, uint32_t oct, std::vector<rtx_entry>& out) {
    out.clear();
    out.reserve(t.n_internal + t.unit_entries.size());
    struct Frame {
        int32_t node;   // SAH node, or -1 - unit
        int64_t close;  // >= 0: the entry whose escape this frame closes
    };
    std::vector<Frame> st{{t.root, -1}};
    while (!st.empty()) {
        const Frame f = st.back();
        st.pop_back();
        if (f.close >= 0) {
            const int32_t esc = (int32_t)out.size();
            std::memcpy(&out[(size_t)f.close].a[3], &esc, 4);
            continue;
        }
        if (f.node < 0) {  // a unit: its entries, the leaf node's escape moved with it
            const uint32_t u = (uint32_t)(-1 - f.node);
            const uint32_t base = (uint32_t)out.size();
            for (uint32_t k = t.unit_first[u]; k < t.unit_first[u + 1]; ++k) out.push_back(t.unit_entries[k]);
            if (t.guarded) {
                const int32_t esc = (int32_t)out.size();
                std::memcpy(&out[base].a[3], &esc, 4);
            }
            continue;
        }
        const rtx_bvh_node& n = t.nodes[f.node];
        rtx_entry e;
        std::memset(&e, 0, sizeof(e));
        for (int k = 0; k < 3; ++k) {
            e.a[k] = n.bmin[k];
            e.b[k] = n.bmax[k];
        }
        const int32_t tag = RTX_E_NODE;
        std::memcpy(&e.b[3], &tag, 4);
        const int64_t me = (int64_t)out.size();
        out.push_back(e);
        int32_t kid[2];
        for (int c = 0; c < 2; ++c) {
            const int32_t cu = t.child_unit[2 * f.node + c];
            kid[c] = cu >= 0 ? -1 - cu : (c == 0 ? n.left : n.right);
        }
        const bool flip = (oct >> t.axis[f.node]) & 1u;  // the near child first
        st.push_back({0, me});
        st.push_back({kid[flip ? 0 : 1], -1});
        st.push_back({kid[flip ? 1 : 0], -1});
    }
}

uint32_t camera_octant(const rtx_camera& c) {
    uint32_t o = 0;
    for (int k = 0; k < 3; ++k) {
        const double f = (double)c.pixel00[k] + (double)c.pixel_du[k] * (0.5 * c.image_width) +
                         (double)c.pixel_dv[k] * (0.5 * c.image_height) - (double)c.center[k];
        if (f < 0.0) o |= 1u << k;
    }
    return o;
}

}  // namespace rtxd
