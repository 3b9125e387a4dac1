// rtx_collapse.hip — the collapsed walk (host code; see rtx_collapse.h).
#include "rtx_collapse.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace rtxd {
namespace {

int32_t tag_of(const rtx_entry& e) {
    int32_t t;
    std::memcpy(&t, &e.b[3], 4);
    return t;
}
int32_t escape_of(const rtx_entry& e) {
    int32_t t;
    std::memcpy(&t, &e.a[3], 4);
    return t;
}

// InBoundary on all three axes (bvh.go:52-61, 84-102).
bool box_passes(const rtx_entry& e, const float o[3], const float d[3], float tmin, float tmax) {
    for (int k = 0; k < 3; ++k) {
        const float inv = 1.0f / d[k];
        float t0 = (e.a[k] - o[k]) * inv, t1 = (e.b[k] - o[k]) * inv;
        if (inv < 0.0f) std::swap(t0, t1);
        if (t0 > tmin) tmin = t0;
        if (t1 < tmax) tmax = t1;
        if (!(tmin < tmax)) return false;
    }
    return true;
}

struct SampleHit {
    float t;
    float n[3];
};

// One closest-hit walk of the threaded layout (an estimate: double-precision primitive tests),
// counting the node entries whose box passes.
bool sample_walk(const std::vector<rtx_entry>& E, const std::vector<float>& quadtab, const float o[3], const float d[3],
                 std::vector<double>& pass, SampleHit& h) {
    float closest = INFINITY;
    bool hit = false;
    const size_t n = E.size();
    for (size_t i = 0; i < n;) {
        const rtx_entry& e = E[i];
        const int32_t tag = tag_of(e);
        if (tag == RTX_E_NODE) {
            if (box_passes(e, o, d, 0.001f, closest)) {
                pass[i] += 1.0;
                ++i;
            } else {
                const int32_t esc = escape_of(e);
                i = esc > (int32_t)i ? (size_t)esc : n;  // (escapes point forward)
            }
            continue;
        }
        ++i;
        if (tag == RTX_E_QUAD) {
            int32_t q;
            std::memcpy(&q, &e.b[0], 4);
            if (q < 0 || (size_t)q * 16 + 16 > quadtab.size()) continue;
            const float* Q = &quadtab[(size_t)q * 16];
            const double nd = (double)e.a[0] * d[0] + (double)e.a[1] * d[1] + (double)e.a[2] * d[2];
            if (std::fabs(nd) < 1e-8) continue;
            const double t = ((double)e.a[3] - ((double)e.a[0] * o[0] + (double)e.a[1] * o[1] + (double)e.a[2] * o[2])) / nd;
            if (!(t > 0.001 && t < closest)) continue;
            double php[3];
            for (int k = 0; k < 3; ++k) php[k] = o[k] + t * d[k] - Q[k];
            const float *u = Q + 4, *v = Q + 8, *w = Q + 12;
            const double pv[3] = {php[1] * v[2] - php[2] * v[1], php[2] * v[0] - php[0] * v[2], php[0] * v[1] - php[1] * v[0]};
            const double up[3] = {u[1] * php[2] - u[2] * php[1], u[2] * php[0] - u[0] * php[2], u[0] * php[1] - u[1] * php[0]};
            const double al = w[0] * pv[0] + w[1] * pv[1] + w[2] * pv[2], be = w[0] * up[0] + w[1] * up[1] + w[2] * up[2];
            if (al < 0.0 || al > 1.0 || be < 0.0 || be > 1.0) continue;
            closest = (float)t;
            for (int k = 0; k < 3; ++k) h.n[k] = e.a[k];
            hit = true;
            continue;
        }
        // a sphere (hittables.go:96-128, in double)
        double oc[3], a = 0.0, hb = 0.0, cc = 0.0;
        for (int k = 0; k < 3; ++k) {
            oc[k] = (double)e.a[k] - o[k];
            a += (double)d[k] * d[k];
            hb += (double)d[k] * oc[k];
            cc += oc[k] * oc[k];
        }
        cc -= (double)e.a[3] * e.a[3];
        const double disc = hb * hb - a * cc;
        if (disc < 0.0 || a == 0.0) continue;
        const double sq = std::sqrt(disc);
        double t = (hb - sq) / a;
        if (!(t > 0.001 && t < closest)) t = (hb + sq) / a;
        if (!(t > 0.001 && t < closest)) continue;
        closest = (float)t;
        const double r = e.a[3] != 0.0f ? (double)e.a[3] : 1.0;
        for (int k = 0; k < 3; ++k) h.n[k] = (float)((o[k] + t * d[k] - e.a[k]) / r);
        hit = true;
    }
    h.t = closest;
    return hit;
}

uint64_t next_u64(uint64_t& s) {  // xorshift64*
    s ^= s >> 12;
    s ^= s << 25;
    s ^= s >> 27;
    return s * 2685821657736338717ull;
}
float unit_float(uint64_t& s) { return (float)((next_u64(s) >> 40) * (1.0 / 16777216.0)); }

// Whether node entry c's box lies inside node entry p's (false on any NaN coordinate).  Trees built
// by NewBVH always nest (NewAabbFromBoxes); a caller's hand-made table need not, and a node whose
// children stick out keeps its test.
bool box_inside(const rtx_entry& c, const rtx_entry& p) {
    for (int k = 0; k < 3; ++k)
        if (!(c.a[k] >= p.a[k] && c.b[k] <= p.b[k])) return false;
    return true;
}

}  // namespace

void sample_node_passes(const std::vector<rtx_entry>& E, const std::vector<float>& quadtab, const rtx_camera& cam,
                        std::vector<double>& pass, double* walks) {
    pass.assign(E.size(), 0.0);
    *walks = 0.0;
    if (E.empty() || cam.image_width == 0 || cam.image_height == 0) return;
    // 64 columns of the image, rows in proportion; two paths per point, up to 4 segments each
    // (randSpheres averages 2.9 segments per sample)
    const char* env = std::getenv("RTX_PLAN_GRID");  // (A/B of the sample size)
    const uint32_t gx = env ? (uint32_t)std::max(1l, std::min(1024l, std::strtol(env, nullptr, 10))) : 64u;
    uint32_t gy = (uint32_t)std::lround((double)gx * cam.image_height / cam.image_width);
    gy = gy < 1 ? 1 : (gy > gx ? gx : gy);
    uint64_t rng = 0x9E3779B97F4A7C15ull;
    for (uint32_t yi = 0; yi < gy; ++yi)
        for (uint32_t xi = 0; xi < gx; ++xi)
            for (int path = 0; path < 2; ++path) {
                const float px = ((float)xi + unit_float(rng)) * cam.image_width / gx - 0.5f;
                const float py = ((float)yi + unit_float(rng)) * cam.image_height / gy - 0.5f;
                float o[3], d[3];
                for (int k = 0; k < 3; ++k) {
                    o[k] = cam.center[k];
                    d[k] = cam.pixel00[k] + px * cam.pixel_du[k] + py * cam.pixel_dv[k] - cam.center[k];
                }
                for (int seg = 0; seg < 4; ++seg) {
                    SampleHit h;
                    *walks += 1.0;
                    if (!sample_walk(E, quadtab, o, d, pass, h)) break;
                    float nd = h.n[0] * d[0] + h.n[1] * d[1] + h.n[2] * d[2];
                    const float sg = nd > 0.0f ? -1.0f : 1.0f;
                    float r[3], l2;
                    do {  // a random unit vector (rejection in the cube)
                        for (int k = 0; k < 3; ++k) r[k] = 2.0f * unit_float(rng) - 1.0f;
                        l2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
                    } while (!(l2 > 1e-6f && l2 <= 1.0f));
                    const float il = 1.0f / std::sqrt(l2);
                    for (int k = 0; k < 3; ++k) {
                        o[k] = o[k] + h.t * d[k];
                        d[k] = sg * h.n[k] + r[k] * il;
                    }
                    if (std::fabs(d[0]) + std::fabs(d[1]) + std::fabs(d[2]) < 1e-6f)
                        for (int k = 0; k < 3; ++k) d[k] = sg * h.n[k];
                }
            }
}

bool collapse_layout(const std::vector<rtx_entry>& E, const std::vector<double>& pass, double walks, bool allow_drop,
                     std::vector<rtx_entry>& out, std::vector<uint8_t>& skip, std::vector<double>* reads) {
    const size_t n = E.size();
    std::vector<int32_t> parent(n, -1);
    std::vector<uint32_t> depth(n, 0), kids(n, 0);
    std::vector<uint8_t> prim_child(n, 0), is_node(n, 0), sticks_out(n, 0);
    uint64_t cells = 0;
    uint32_t n_nodes = 0;
    {
        std::vector<std::pair<uint32_t, uint32_t>> open;  // (node entry, escape)
        for (size_t i = 0; i < n; ++i) {
            while (!open.empty() && open.back().second <= i) open.pop_back();
            if (!open.empty()) {
                parent[i] = (int32_t)open.back().first;
                ++kids[open.back().first];
            }
            if (tag_of(E[i]) == RTX_E_NODE) {
                is_node[i] = 1;
                if (parent[i] >= 0 && !box_inside(E[i], E[parent[i]])) sticks_out[parent[i]] = 1;
                depth[i] = (uint32_t)open.size();
                cells += depth[i] + 1;
                ++n_nodes;
                const int32_t esc = escape_of(E[i]);
                open.push_back({(uint32_t)i, esc > (int32_t)i ? (uint32_t)esc : (uint32_t)n});
            } else if (parent[i] >= 0) {
                prim_child[parent[i]] = 1;
            }
        }
    }
    skip.assign(n_nodes, 0);
    if (reads) reads->clear();
    if (cells > (64ull << 20) || pass.size() != n) {
        out = E;
        return false;
    }
    // cost[i][j]: box tests of node i's subtree when its nearest kept ancestor is the one at depth
    // j - 1 (j = 0: none; the walk's start, `walks` times).  Children finish before their parent
    // (pre-order, walked backwards) and fold their tables into the parent's sums.
    std::vector<double> acc_keep(n, 0.0);
    std::vector<std::vector<double>> acc_drop(n);
    std::vector<std::vector<uint8_t>> keep(n);
    std::vector<double> counts, cost;
    for (size_t ii = n; ii-- > 0;) {
        if (!is_node[ii]) continue;
        const uint32_t d = depth[ii];
        counts.assign(d + 1, walks);
        for (int32_t y = parent[ii]; y >= 0; y = parent[y]) counts[depth[y] + 1] = pass[y];
        const bool collapsible = allow_drop && kids[ii] > 0 && !prim_child[ii] && !sticks_out[ii];
        std::vector<double>& drop = acc_drop[ii];
        if (drop.size() < d + 1) drop.resize(d + 1, 0.0);
        cost.assign(d + 1, 0.0);
        keep[ii].assign(d + 1, 1);
        for (uint32_t j = 0; j <= d; ++j) {
            const double k = counts[j] + acc_keep[ii];
            if (collapsible && drop[j] < k) {
                cost[j] = drop[j];
                keep[ii][j] = 0;
            } else {
                cost[j] = k;
            }
        }
        std::vector<double>().swap(drop);
        const int32_t p = parent[ii];
        if (p >= 0) {
            const uint32_t dp = depth[p];
            acc_keep[p] += cost[dp + 1];
            std::vector<double>& pd = acc_drop[p];
            if (pd.size() < dp + 1) pd.resize(dp + 1, 0.0);
            for (uint32_t j = 0; j <= dp; ++j) pd[j] += cost[j];
        }
    }
    // decisions, top down: jn[i] = the j its children see
    std::vector<uint32_t> jn(n, 0);
    std::vector<uint8_t> drop_entry(n, 0);
    uint32_t ord = 0;
    for (size_t i = 0; i < n; ++i) {
        if (!is_node[i]) continue;
        const uint32_t j = parent[i] >= 0 ? jn[parent[i]] : 0u;
        const bool k = keep[i][j] != 0;
        jn[i] = k ? depth[i] + 1 : j;
        drop_entry[i] = k ? 0 : 1;
        skip[ord++] = drop_entry[i];
    }
    std::vector<uint32_t> map(n + 1);
    uint32_t m = 0;
    for (size_t i = 0; i < n; ++i) {
        map[i] = m;
        if (!drop_entry[i]) ++m;
    }
    map[n] = m;
    out.clear();
    out.reserve(m);
    if (reads) reads->reserve(m);
    for (size_t i = 0; i < n; ++i) {
        if (drop_entry[i]) continue;
        if (reads) {  // estimated reads of the entry: the passes of its nearest kept ancestor
            const uint32_t j = parent[i] >= 0 ? jn[parent[i]] : 0u;
            int32_t y = parent[i];
            while (y >= 0 && depth[y] + 1 > j) y = parent[y];
            reads->push_back(j == 0 || y < 0 ? walks : pass[y]);
        }
        rtx_entry e = E[i];
        if (is_node[i]) {
            const int32_t esc = escape_of(e);
            const int32_t ne = (int32_t)map[esc >= 0 && (size_t)esc <= n ? (size_t)esc : n];
            std::memcpy(&e.a[3], &ne, 4);
        }
        out.push_back(e);
    }
    return true;
}

}  // namespace rtxd
