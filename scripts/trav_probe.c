/* trav_probe.c — measurement tool (not product code): how many box and primitive tests a
 * segment costs under other traversal orders of the reference's own BVH, on the paths the
 * reference takes.  Every segment is traced by the oracle (world_hit, bvh.go:220-249: left,
 * then right clipped to the left hit), and the same ray is walked again under:
 *   oct  : near child first, the near child chosen per node from the sign of the ray's
 *          direction along the axis that separates the children's centres most (one
 *          threaded order per direction octant: stackless on the GPU);
 *   dist : both children's boxes tested at the parent, the nearer entry walked first, the
 *          other pushed with its entry distance and skipped on pop if past the closest hit.
 * The closest hit (t, primitive) of every order is checked against the reference's.
 *
 *   make -C scripts trav_probe && scripts/trav_probe random_spheres 192 8
 */
#include "../oracle/oracle.c"

#include "../include/rtx_host.h"

typedef struct {
    uint64_t box, prim, mism_t, mism_prim, segs;
} probe_t;

static int ref_prim_hit(const rtx_scene_desc* s, int32_t ref, const ray_t* r, float tmin, float tmax, float* t) {
    hit_t h;
    uint32_t p = (uint32_t)(~ref), type = p >> 28, idx = p & 0x0FFFFFFFu;
    int ok = type == RTX_PRIM_QUAD ? quad_hit(&s->quads[idx], r, tmin, tmax, &h)
                                   : sphere_hit(NULL, &s->spheres[idx], r, tmin, tmax, &h, 0);
    if (ok) *t = h.t;
    return ok;
}

static float centre(const rtx_scene_desc* s, int32_t ref, int ax) {
    if (ref >= 0) return 0.5f * (s->nodes[ref].bmin[ax] + s->nodes[ref].bmax[ax]);
    uint32_t p = (uint32_t)(~ref), type = p >> 28, idx = p & 0x0FFFFFFFu;
    if (type == RTX_PRIM_SPHERE) return s->spheres[idx].center[ax];
    const rtx_quad* q = &s->quads[idx];
    float u[3] = {q->u[0], q->u[1], q->u[2]}, v[3] = {q->v[0], q->v[1], q->v[2]};
    return q->q[ax] + 0.5f * (u[ax] + v[ax]);
}

/* Does the ray visit `first` before `second` (oct mode)? */
static int near_first(const rtx_scene_desc* s, int32_t a, int32_t b, const ray_t* r) {
    int best = 0;
    float bd = -1.0f;
    for (int ax = 0; ax < 3; ++ax) {
        float d = fabsf(centre(s, a, ax) - centre(s, b, ax));
        if (d > bd) { bd = d; best = ax; }
    }
    float dir = best == 0 ? r->dir.x : (best == 1 ? r->dir.y : r->dir.z);
    float ca = centre(s, a, best), cb = centre(s, b, best);
    return dir >= 0.0f ? ca <= cb : ca >= cb;
}

/* slab entry of a node box (InBoundary), or +inf on a miss */
static float box_entry(const rtx_bvh_node* n, const ray_t* r, float tmin, float tmax) {
    if (in_boundary(r->dir.x, r->origin.x, n->bmin[0], n->bmax[0], &tmin, &tmax))
        if (in_boundary(r->dir.y, r->origin.y, n->bmin[1], n->bmax[1], &tmin, &tmax))
            if (in_boundary(r->dir.z, r->origin.z, n->bmin[2], n->bmax[2], &tmin, &tmax)) return tmin;
    return INFINITY;
}

static void oct_walk(const rtx_scene_desc* s, int32_t ref, const ray_t* r, float* closest, int32_t* hit, probe_t* p) {
    if (ref >= 0) {
        const rtx_bvh_node* n = &s->nodes[ref];
        p->box++;
        if (!aabb_hit(n, r, 0.001f, *closest)) return;
        if (n->left == n->right) { oct_walk(s, n->left, r, closest, hit, p); return; }
        if (near_first(s, n->left, n->right, r)) {
            oct_walk(s, n->left, r, closest, hit, p);
            oct_walk(s, n->right, r, closest, hit, p);
        } else {
            oct_walk(s, n->right, r, closest, hit, p);
            oct_walk(s, n->left, r, closest, hit, p);
        }
        return;
    }
    p->prim++;
    float t;
    if (ref_prim_hit(s, ref, r, 0.001f, *closest, &t)) { *closest = t; *hit = ref; }
}

static void dist_walk(const rtx_scene_desc* s, int32_t root, const ray_t* r, float* closest, int32_t* hit, probe_t* p) {
    struct { int32_t ref; float t; } st[128];
    int sp = 0;
    if (root >= 0) {
        p->box++;
        float t = box_entry(&s->nodes[root], r, 0.001f, *closest);
        if (t == INFINITY) return;
    }
    st[sp].ref = root; st[sp].t = 0.0f; ++sp;
    while (sp) {
        --sp;
        int32_t ref = st[sp].ref;
        if (st[sp].t >= *closest) continue;
        if (ref < 0) {
            p->prim++;
            float t;
            if (ref_prim_hit(s, ref, r, 0.001f, *closest, &t)) { *closest = t; *hit = ref; }
            continue;
        }
        const rtx_bvh_node* n = &s->nodes[ref];
        int32_t c[2] = {n->left, n->right};
        int nc = n->left == n->right ? 1 : 2;
        float te[2];
        for (int k = 0; k < nc; ++k) {
            if (c[k] >= 0) { p->box++; te[k] = box_entry(&s->nodes[c[k]], r, 0.001f, *closest); }
            else te[k] = 0.0f; /* a primitive child: tested when popped */
        }
        if (nc == 2 && te[1] < te[0]) { int32_t x = c[0]; c[0] = c[1]; c[1] = x; float y = te[0]; te[0] = te[1]; te[1] = y; }
        for (int k = nc - 1; k >= 0; --k)
            if (te[k] != INFINITY) { st[sp].ref = c[k]; st[sp].t = te[k]; ++sp; }
    }
}


/* ---- a binned-SAH tree over the reference tree's primitives (sphere scenes) ---------- */
typedef struct { float mn[3], mx[3]; int32_t l, r; int32_t first, count; } snode_t; /* count > 0: leaf */
static snode_t* SN; static int n_sn; static int32_t* SP; /* prims (refs) in leaf order */
static int sah_leaf = 1;
static int guard = 0;
static int32_t* GUARD_OF; /* guard 3: sphere -> its reference leaf node */
static float INFL = 0.02f;
static int FAR; static float RN = 1e30f; static uint64_t n_far;
static float c_isect = 1.5f;

static aabb_t prim_box(const rtx_scene_desc* s, int32_t ref) {
    uint32_t p = (uint32_t)(~ref), idx = p & 0x0FFFFFFFu;
    return sphere_bounds(&s->spheres[idx]);
}
static float area(aabb_t b) {
    float dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
    return dx * dy + dy * dz + dz * dx;
}
static aabb_t empty_box(void) { aabb_t b = {{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}}; return b; }
static aabb_t* PB; static float* PC; /* per prim slot: box, centroid x3 */

static int sah_build(const rtx_scene_desc* s, int first, int count) {
    int me = n_sn++;
    aabb_t b = empty_box(), cb = empty_box();
    for (int i = first; i < first + count; ++i) {
        b = box_union(b, PB[i]);
        for (int k = 0; k < 3; ++k) { if (PC[3*i+k] < cb.mn[k]) cb.mn[k] = PC[3*i+k]; if (PC[3*i+k] > cb.mx[k]) cb.mx[k] = PC[3*i+k]; }
    }
    memcpy(SN[me].mn, b.mn, 12); memcpy(SN[me].mx, b.mx, 12);
    SN[me].count = 0;
    enum { NB = 32 };
    float best = INFINITY; int bax = -1, bsplit = -1;
    if (count > 1) {
        for (int ax = 0; ax < 3; ++ax) {
            float lo = cb.mn[ax], ext = cb.mx[ax] - cb.mn[ax];
            if (!(ext > 0)) continue;
            aabb_t bb[NB]; int bc[NB];
            for (int k = 0; k < NB; ++k) { bb[k] = empty_box(); bc[k] = 0; }
            for (int i = first; i < first + count; ++i) {
                int k = (int)((PC[3*i+ax] - lo) / ext * NB); if (k >= NB) k = NB - 1; if (k < 0) k = 0;
                bb[k] = box_union(bb[k], PB[i]); bc[k]++;
            }
            float ra[NB]; int rc[NB]; aabb_t acc = empty_box(); int n = 0;
            for (int k = NB - 1; k > 0; --k) { acc = box_union(acc, bb[k]); n += bc[k]; ra[k] = area(acc); rc[k] = n; }
            acc = empty_box(); n = 0;
            for (int k = 0; k < NB - 1; ++k) {
                acc = box_union(acc, bb[k]); n += bc[k];
                if (n == 0 || rc[k+1] == 0) continue;
                float c = area(acc) * n + ra[k+1] * rc[k+1];
                if (c < best) { best = c; bax = ax; bsplit = k; }
            }
        }
    }
    float leaf_cost = c_isect * count * area(b);
    float split_cost = area(b) + c_isect * best; /* 1 box test for the node, then the children */
    if (count <= sah_leaf && (bax < 0 || leaf_cost <= split_cost || count == 1)) {
        SN[me].first = first; SN[me].count = count; return me;
    }
    if (bax < 0) { /* all centres equal: split in the middle */
        bsplit = -1;
    }
    int mid;
    if (bsplit >= 0) {
        float lo = cb.mn[bax], ext = cb.mx[bax] - cb.mn[bax];
        int i = first, j = first + count - 1;
        while (i <= j) {
            int k = (int)((PC[3*i+bax] - lo) / ext * NB); if (k >= NB) k = NB - 1; if (k < 0) k = 0;
            if (k <= bsplit) ++i;
            else { aabb_t tb = PB[i]; PB[i] = PB[j]; PB[j] = tb; for (int q = 0; q < 3; ++q) { float tc = PC[3*i+q]; PC[3*i+q] = PC[3*j+q]; PC[3*j+q] = tc; } int32_t tr = SP[i]; SP[i] = SP[j]; SP[j] = tr; --j; }
        }
        mid = i;
        if (mid == first || mid == first + count) mid = first + count / 2;
    } else mid = first + count / 2;
    int l = sah_build(s, first, mid - first);
    int r = sah_build(s, mid, first + count - mid);
    SN[me].l = l; SN[me].r = r;
    return me;
}

static void sah_walk(const rtx_scene_desc* s, int ni, const ray_t* r, float* closest, probe_t* p, int oct) {
    const snode_t* n = &SN[ni];
    p->box++;
    rtx_bvh_node bn; memcpy(bn.bmin, n->mn, 12); memcpy(bn.bmax, n->mx, 12);
    if (!aabb_hit(&bn, r, 0.001f, *closest)) return;
    if (n->count) {
        for (int i = n->first; i < n->first + n->count; ++i) {
            int32_t pr[2] = {SP[i], SP[i]};
            int np = 1;
            if (guard == 4) { /* own inflated box only */ }
            else if (guard == 3) {  /* the sphere's reference leaf box, then the sphere */
                const rtx_bvh_node* gb = &s->nodes[GUARD_OF[(~SP[i]) & 0x0FFFFFFF]];
                p->box++;
                if (!aabb_hit(gb, r, 0.001f, *closest)) continue;
            } else if (guard) { const rtx_bvh_node* b = &s->nodes[SP[i]]; pr[0] = b->left; pr[1] = b->right; np = b->left == b->right ? 1 : 2; }
            for (int q = 0; q < np; ++q) {
                p->prim++;
                float t;
                if (ref_prim_hit(s, pr[q], r, 0.001f, *closest, &t)) *closest = t;
            }
        }
        return;
    }
    int a = n->l, b = n->r;
    static int ord = -1;
    if (ord < 0) ord = getenv("ORD") ? atoi(getenv("ORD")) : 0;
    if (!oct && ord) {
        aabb_t ba, bb; memcpy(ba.mn, SN[a].mn, 12); memcpy(ba.mx, SN[a].mx, 12); memcpy(bb.mn, SN[b].mn, 12); memcpy(bb.mx, SN[b].mx, 12);
        int sw = ord == 1 ? 1 : (ord == 2 ? area(ba) < area(bb) : area(ba) > area(bb));
        if (ord == 4) { /* near-first along the camera's forward direction (the split axis of the node) */
            extern float CAMF[3];
            int best = 0; float bd = -1;
            for (int ax = 0; ax < 3; ++ax) { float d = fabsf((SN[a].mn[ax] + SN[a].mx[ax]) - (SN[b].mn[ax] + SN[b].mx[ax])); if (d > bd) { bd = d; best = ax; } }
            float ca = SN[a].mn[best] + SN[a].mx[best], cb2 = SN[b].mn[best] + SN[b].mx[best];
            sw = CAMF[best] >= 0.0f ? ca > cb2 : ca < cb2;
        }
        if (sw) { int t = a; a = b; b = t; }
    }
    if (oct) {
        int best = 0; float bd = -1;
        for (int ax = 0; ax < 3; ++ax) { float d = fabsf((SN[a].mn[ax] + SN[a].mx[ax]) - (SN[b].mn[ax] + SN[b].mx[ax])); if (d > bd) { bd = d; best = ax; } }
        float dir = best == 0 ? r->dir.x : (best == 1 ? r->dir.y : r->dir.z);
        float ca = SN[a].mn[best] + SN[a].mx[best], cb2 = SN[b].mn[best] + SN[b].mx[best];
        if (dir >= 0.0f ? ca > cb2 : ca < cb2) { int t = a; a = b; b = t; }
    }
    sah_walk(s, a, r, closest, p, oct);
    sah_walk(s, b, r, closest, p, oct);
}
float CAMF[3];
static probe_t P_sah, P_saho;
static void sah_probe(const rtx_scene_desc* s, const ray_t* r, float t_ref) {
    for (int m = 0; m < 2; ++m) {
        probe_t* p = m ? &P_saho : &P_sah;
        float closest = INFINITY;
        sah_walk(s, 0, r, &closest, p, m);
        if (!(closest == t_ref || (closest != closest && t_ref != t_ref))) {
            p->mism_t++;
            if (getenv("VERBOSE")) fprintf(stderr, "mismatch: o=(%a,%a,%a) d=(%a,%a,%a) ref t=%.9g sah t=%.9g\n", r->origin.x, r->origin.y,
                r->origin.z, r->dir.x, r->dir.y, r->dir.z, t_ref, closest);
            if (getenv("VERBOSE")) for (uint32_t q = 0; q < s->n_spheres; ++q) {
                float t; int32_t ref = RTX_REF_PRIM(RTX_PRIM_SPHERE, q);
                if (ref_prim_hit(s, ref, r, 0.001f, INFINITY, &t) && t < 14.8f) {
                    aabb_t b = sphere_bounds(&s->spheres[q]); rtx_bvh_node bn; memcpy(bn.bmin, b.mn, 12); memcpy(bn.bmax, b.mx, 12);
                    fprintf(stderr, "  sphere %u c=(%.9g %.9g %.9g) r=%.9g t=%.9g own-box hit=%d\n", q, s->spheres[q].center[0], s->spheres[q].center[1], s->spheres[q].center[2], s->spheres[q].radius, t, aabb_hit(&bn, r, 0.001f, INFINITY));
                }
            }
        }
    }
}
/* guard: 1: the SAH units are the reference tree's leaves (nodes of 1-2 primitives), with their boxes */
static void sah_setup(const rtx_scene_desc* s) {
    int n = (int)s->n_spheres;
    if (guard == 3 || guard == 4) {  /* single spheres, navigation boxes = own boxes inflated by INFL (4: no leaf check) */
        GUARD_OF = malloc(n * 4);
        for (uint32_t i = 0; i < s->n_nodes; ++i) {
            const rtx_bvh_node* b = &s->nodes[i];
            if (b->left < 0) GUARD_OF[(~b->left) & 0x0FFFFFFF] = (int32_t)i;
            if (b->right < 0) GUARD_OF[(~b->right) & 0x0FFFFFFF] = (int32_t)i;
        }
        SN = calloc(2 * n + 1, sizeof(snode_t)); SP = malloc(n * 4); PB = malloc(n * sizeof(aabb_t)); PC = malloc(12 * n);
        for (int i = 0; i < n; ++i) {
            SP[i] = RTX_REF_PRIM(RTX_PRIM_SPHERE, i); PB[i] = prim_box(s, SP[i]);
            for (int k = 0; k < 3; ++k) { PB[i].mn[k] -= INFL; PB[i].mx[k] += INFL; PC[3*i+k] = s->spheres[i].center[k]; }
        }
        sah_build(s, 0, n);
        return;
    }
    if (guard) {
        int m = 0;
        SN = calloc(2 * n + 1, sizeof(snode_t)); SP = malloc(n * 4); PB = malloc(n * sizeof(aabb_t)); PC = malloc(12 * n);
        for (uint32_t i = 0; i < s->n_nodes; ++i) {
            const rtx_bvh_node* b = &s->nodes[i];
            if (b->left >= 0 || b->right >= 0) continue;
            SP[m] = (int32_t)i;
            memcpy(PB[m].mn, b->bmin, 12); memcpy(PB[m].mx, b->bmax, 12);
            for (int k = 0; k < 3; ++k) PC[3*m+k] = 0.5f * (b->bmin[k] + b->bmax[k]);
            ++m;
        }
        sah_build(s, 0, m);
        return;
    }
    SN = calloc(2 * n + 1, sizeof(snode_t)); SP = malloc(n * 4); PB = malloc(n * sizeof(aabb_t)); PC = malloc(12 * n);
    for (int i = 0; i < n; ++i) {
        SP[i] = RTX_REF_PRIM(RTX_PRIM_SPHERE, i); PB[i] = prim_box(s, SP[i]);
        for (int k = 0; k < 3; ++k) PC[3*i+k] = s->spheres[i].center[k];
    }
    sah_build(s, 0, n);
}

static probe_t P_oct, P_dist;
static uint64_t probe_ref_box, probe_ref_prim, segs;

static uint64_t far_hist[8]; /* segments whose origin lies > 0/5/10/20/40/80/160/inf units outside the core box */
static float CORE_MN[3] = {-11.2f, 0.0f, -11.2f}, CORE_MX[3] = {11.2f, 2.0f, 11.2f};
static void probe_segment(const ctx_t* cx, const ray_t* r, int hit_any, const hit_t* h) {
    const rtx_scene_desc* s = cx->s;
    {
        float o[3] = {r->origin.x, r->origin.y, r->origin.z}, dm = 0;
        for (int k = 0; k < 3; ++k) { float e = o[k] < CORE_MN[k] ? CORE_MN[k] - o[k] : (o[k] > CORE_MX[k] ? o[k] - CORE_MX[k] : 0); if (e > dm) dm = e; }
        const float lim[7] = {0, 5, 10, 20, 40, 80, 160};
        int b = 7; for (int q = 0; q < 7; ++q) if (dm <= lim[q]) { b = q; break; }
        far_hist[b]++;
    }
    float t_ref = hit_any ? h->t : INFINITY;
    {
        float o[3] = {r->origin.x, r->origin.y, r->origin.z}, dm = 0;
        for (int k = 0; k < 3; ++k) { float e = o[k] < CORE_MN[k] ? CORE_MN[k] - o[k] : (o[k] > CORE_MX[k] ? o[k] - CORE_MX[k] : 0); if (e > dm) dm = e; }
        FAR = dm > RN;
        if (FAR) { n_far++; return; }
    }
    for (int m = 0; m < 2; ++m) {
        probe_t* p = m ? &P_dist : &P_oct;
        float closest = INFINITY;
        int32_t hit = 0;
        for (uint32_t i = 0; i < s->n_roots; ++i) {
            if (m) dist_walk(s, s->roots[i], r, &closest, &hit, p);
            else oct_walk(s, s->roots[i], r, &closest, &hit, p);
        }
        if (!(closest == t_ref || (closest != closest && t_ref != t_ref))) p->mism_t++;
        (void)hit;
    }
    sah_probe(s, r, t_ref);
}

static uint64_t n_far_paths, n_paths, n_far_before;
static vec3 probe_color(const ctx_t* cx, ray_t r, rng_t* rng, int depth) {
    vec3 thr = v3(1.0f, 1.0f, 1.0f), acc = v3(0.0f, 0.0f, 0.0f);
    n_paths++; n_far_before = n_far;
    struct F { uint64_t* a; uint64_t b; } fin = {&n_far_paths, 0}; (void)fin;
    for (; depth > 0; --depth) {
        hit_t h;
        cx->c->segments++;
        uint64_t nv = cx->c->node_visits, pt = cx->c->prim_tests;
        int hit_any = world_hit(cx, &r, 0.001f, INFINITY, &h);
        probe_ref_box += cx->c->node_visits - nv;
        probe_ref_prim += cx->c->prim_tests - pt;
        segs++;
        probe_segment(cx, &r, hit_any, &h);
        if (n_far_before != (uint64_t)-1 && n_far != n_far_before) { n_far_paths++; n_far_before = (uint64_t)-1; }
        if (!hit_any) return acc;
        int has_emit;
        vec3 emit = material_emit(cx, &h, &has_emit);
        if (has_emit) acc = v_add(acc, v_mul(thr, emit));
        vec3 att;
        ray_t sc;
        rng_event(rng, cx->cam->max_depth - (uint32_t)depth + 1u);
        if (!material_scatter(cx, &r, &h, rng, &att, &sc)) return acc;
        thr = v_mul(thr, att);
        r = sc;
    }
    return acc;
}

int main(int argc, char** argv) {
    const char* name = argc > 1 ? argv[1] : "random_spheres";
    int width = argc > 2 ? atoi(argv[2]) : 192;
    int spp = argc > 3 ? atoi(argv[3]) : 4;
    int stride = argc > 4 ? atoi(argv[4]) : 1;
    rtxhost_scene* hs = NULL;
    if (rtxhost_build_scene(name, 1, &hs)) { fprintf(stderr, "%s\n", rtxhost_last_error()); return 1; }
    const rtx_scene_desc* s = rtxhost_scene_desc(hs);
    rtx_camera cam;
    if (getenv("GUARD")) guard = atoi(getenv("GUARD"));
    if (getenv("INFL")) INFL = atof(getenv("INFL"));
    if (getenv("RN")) RN = atof(getenv("RN"));
    if (getenv("LEAF")) sah_leaf = atoi(getenv("LEAF"));
    if (getenv("CI")) c_isect = atof(getenv("CI"));
    sah_setup(s);
    rtxhost_scene_camera(hs, width, spp, 0, &cam);
    for (int k = 0; k < 3; ++k) CAMF[k] = cam.pixel00[k] + cam.pixel_du[k] * cam.image_width * 0.5f + cam.pixel_dv[k] * cam.image_height * 0.5f - cam.center[k];
    oracle_counters c;
    memset(&c, 0, sizeof(c));
    ctx_t cx = {s, &cam, 7, ORACLE_ORDER_ITERATIVE, &c};
    for (uint32_t j = 0; j < cam.image_height; j += stride)
        for (uint32_t i = 0; i < cam.image_width; i += stride)
            for (uint32_t k = 0; k < cam.samples_per_pixel; ++k) {
                rng_t rng;
                rng.key[0] = 7; rng.key[1] = 0;
                rng.pixel = j * cam.image_width + i; rng.sample = k;
                rng.event = rng.attempt = rng.word = 0;
                rng.draws = &c.rng_draws;
                ray_t r = get_ray(&cx, &rng, i, j);
                probe_color(&cx, r, &rng, (int)cam.max_depth);
            }
    printf("%s %ux%u x%u spp (stride %d): %llu segments\n", name, cam.image_width, cam.image_height,
           cam.samples_per_pixel, stride, (unsigned long long)segs);
    printf("  ref : box %.2f prim %.2f per segment\n", (double)probe_ref_box / segs, (double)probe_ref_prim / segs);
    printf("  oct : box %.2f prim %.2f per segment, t mismatches %llu\n", (double)P_oct.box / segs,
           (double)P_oct.prim / segs, (unsigned long long)P_oct.mism_t);
    printf("  dist: box %.2f prim %.2f per segment, t mismatches %llu\n", (double)P_dist.box / segs,
           (double)P_dist.prim / segs, (unsigned long long)P_dist.mism_t);
    printf("  origin outside the core box by <=0/5/10/20/40/80/160/more:");
    for (int q = 0; q < 8; ++q) printf(" %.2e", (double)far_hist[q] / segs);
    printf("\n");
    printf("  far segments (origin > RN outside the core box): %.4f\n", (double)n_far / segs);
    segs -= n_far;
    printf("  paths with a far segment: %.4f of %llu\n", (double)n_far_paths / n_paths, (unsigned long long)n_paths);
    printf("  sah : box %.2f prim %.2f per segment, t mismatches %llu (%d nodes, leaf <= %d)\n", (double)P_sah.box / segs,
           (double)P_sah.prim / segs, (unsigned long long)P_sah.mism_t, n_sn, sah_leaf);
    printf("  saho: box %.2f prim %.2f per segment, t mismatches %llu\n", (double)P_saho.box / segs,
           (double)P_saho.prim / segs, (unsigned long long)P_saho.mism_t);
    return 0;
}
