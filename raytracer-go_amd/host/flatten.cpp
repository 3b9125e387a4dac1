// flatten.cpp — walk the Hittable tree by type switch into the rtx.h tables.
//
// This is the step a cgo Render performs before crossing the boundary:
// *BVH -> node (bBox, left, right), *Sphere -> sphere, materials and textures by
// identity (a shared material/texture is stored once).  Nodes are numbered in
// pre-order (a node before its children, left before right), the order NewBVH
// creates them in.  A World passed to Render gives one root per item (its linear
// scan order, hittables.go:55-72).
#include <unordered_map>

#include <cstring>

#include "internal.h"

namespace internal {

namespace {

struct Flattener {
    FlatScene& fs;
    std::unordered_map<const Hittable*, int32_t> refs;
    std::unordered_map<const Material*, uint32_t> mats;
    std::unordered_map<const Texture*, uint32_t> texs;
    Error err;

    explicit Flattener(FlatScene& f) : fs(f) {}

    bool fail(int code, const std::string& msg) {
        if (!err) err = Error{code, msg};
        return false;
    }

    bool texture(const TexturePtr& t, uint32_t& out) {
        if (!t) return fail(RTX_ERR_INVALID_ARG, "nil Texture");
        auto it = texs.find(t.get());
        if (it != texs.end()) { out = it->second; return true; }
        rtx_texture r{};
        if (auto s = dynamic_cast<const SolidColor*>(t.get())) {
            r.type = RTX_TEX_SOLID;
            r.even[0] = s->albedo.X; r.even[1] = s->albedo.Y; r.even[2] = s->albedo.Z;
        } else if (auto c = dynamic_cast<const Checkered*>(t.get())) {
            r.type = RTX_TEX_CHECKERED;
            r.scale = c->scale;
            r.even[0] = c->even.X; r.even[1] = c->even.Y; r.even[2] = c->even.Z;
            r.odd[0] = c->odd.X; r.odd[1] = c->odd.Y; r.odd[2] = c->odd.Z;
        } else if (auto im = dynamic_cast<const ImageTexture*>(t.get())) {
            // At(i, j).RGBA() for the raster, then the border colour (rtx.h RTX_TEX_IMAGE)
            r.type = RTX_TEX_IMAGE;
            const Image* img = im->img.get();
            if (!img) return fail(RTX_ERR_INVALID_ARG, "ImageTexture with a nil image");
            const Rectangle b = img->Bounds();
            if (b.Dy() > 0) {
                // GetTexture indexes At(int(u*Dx), int(v*Dy)) from 0, so the table is exact when
                // the bounds start at the origin (jpeg.Decode, image.New*); others stay on the CPU.
                if (b.MinX != 0 || b.MinY != 0)
                    return fail(RTX_ERR_UNSUPPORTED, "ImageTexture whose Bounds().Min is not (0, 0)");
                if (b.Dx() > 0xFFFFFFF || b.Dy() > 0xFFFFFFF) return fail(RTX_ERR_INVALID_ARG, "image too large");
                r.width = (uint32_t)b.Dx();
                r.height = (uint32_t)b.Dy();
                if (fs.texels.size() & 1u) fs.texels.push_back(0);  // texel_offset even (8-B texels)
                r.texel_offset = (uint32_t)fs.texels.size();
                fs.texels.reserve(fs.texels.size() + 2 * ((size_t)r.width * r.height + 1));
                auto put = [&](const RGBA64& c) {
                    fs.texels.push_back((c.r & 0xFFFFu) | (c.g & 0xFFFFu) << 16);
                    fs.texels.push_back((c.b & 0xFFFFu) | (c.a & 0xFFFFu) << 16);
                };
                for (int64_t j = 0; j < b.Dy(); ++j)
                    for (int64_t i = 0; i < b.Dx(); ++i) put(img->At(i, j));
                put(img->At(b.MaxX, b.MinY));  // outside the bounds
            } else {
                r.width = (uint32_t)std::max<int64_t>(b.Dx(), 0);
                r.height = 0;  // Dy() <= 0: GetTexture's debug colour, no texels
            }
        } else if (auto nt = dynamic_cast<const NoiseTexture*>(t.get())) {  // RTX_NOISE_TEXELS layout
            const Perlin& per = nt->perlin;
            if (per.randVec3.size() != 256 || per.permX.size() != 256 || per.permY.size() != 256 ||
                per.permZ.size() != 256)
                return fail(RTX_ERR_INVALID_ARG, "Perlin tables must hold 256 entries");
            r.type = RTX_TEX_NOISE;
            r.scale = nt->scale;
            r.texel_offset = (uint32_t)fs.texels.size();
            for (const Vec3& g : per.randVec3)
                for (float c : {g.X, g.Y, g.Z}) {
                    uint32_t bits;
                    std::memcpy(&bits, &c, 4);
                    fs.texels.push_back(bits);
                }
            for (const auto* perm : {&per.permX, &per.permY, &per.permZ})
                for (int v : *perm) fs.texels.push_back((uint32_t)v);
        } else {
            return fail(RTX_ERR_UNSUPPORTED, "unknown Texture type");
        }
        out = (uint32_t)fs.textures.size();
        fs.textures.push_back(r);
        texs[t.get()] = out;
        return true;
    }

    bool material(const MaterialPtr& m, uint32_t& out) {
        if (!m) return fail(RTX_ERR_INVALID_ARG, "nil Material");
        auto it = mats.find(m.get());
        if (it != mats.end()) { out = it->second; return true; }
        rtx_material r{};
        if (auto l = dynamic_cast<const Lambertian*>(m.get())) {
            r.type = RTX_MAT_LAMBERTIAN;
            if (!texture(l->albedo, r.texture)) return false;
        } else if (auto me = dynamic_cast<const Metal*>(m.get())) {
            r.type = RTX_MAT_METAL;
            r.albedo[0] = me->albedo.X; r.albedo[1] = me->albedo.Y; r.albedo[2] = me->albedo.Z;
            r.fuzz = me->fuzz;
        } else if (auto d = dynamic_cast<const Dielectric*>(m.get())) {
            r.type = RTX_MAT_DIELECTRIC;
            r.ior = d->refractiveIndex;
        } else if (auto dl = dynamic_cast<const DiffuseLight*>(m.get())) {
            r.type = RTX_MAT_DIFFUSE_LIGHT;
            if (!texture(dl->emit, r.texture)) return false;
        } else {
            return fail(RTX_ERR_UNSUPPORTED, "unknown Material type");
        }
        out = (uint32_t)fs.materials.size();
        fs.materials.push_back(r);
        mats[m.get()] = out;
        return true;
    }

    // Iterative pre-order walk (trees of 1e5+ spheres are ~17 deep, but a hand-built
    // chain could be deep).
    bool ref(const HittablePtr& root, int32_t& out) {
        // child slots live in fs.nodes, which may reallocate: patch through indices
        struct Patch {
            int32_t node;  // side 2: the index into fs.list_refs
            int side;      // 0 left, 1 right, 2 list item, -1 external slot
            int32_t* ext;
        };
        std::vector<std::pair<const Hittable*, Patch>> stack{{root.get(), Patch{-1, -1, &out}}};
        while (!stack.empty()) {
            auto [h, patch] = stack.back();
            stack.pop_back();
            int32_t r;
            if (!h) return fail(RTX_ERR_INVALID_ARG, "nil Hittable");
            auto it = refs.find(h);
            if (it != refs.end()) {
                r = it->second;
            } else if (auto b = dynamic_cast<const BVH*>(h)) {
                r = (int32_t)fs.nodes.size();
                rtx_bvh_node n{};
                n.bmin[0] = b->bBox.x.min; n.bmin[1] = b->bBox.y.min; n.bmin[2] = b->bBox.z.min;
                n.bmax[0] = b->bBox.x.max; n.bmax[1] = b->bBox.y.max; n.bmax[2] = b->bBox.z.max;
                fs.nodes.push_back(n);
                refs[h] = r;
                stack.push_back({b->right.get(), Patch{r, 1, nullptr}});
                stack.push_back({b->left.get(), Patch{r, 0, nullptr}});
            } else if (auto s = dynamic_cast<const Sphere*>(h)) {
                rtx_sphere sp{};
                sp.center[0] = s->Center.X; sp.center[1] = s->Center.Y; sp.center[2] = s->Center.Z;
                sp.radius = s->Radius;
                if (!material(s->Mat, sp.material)) return false;
                r = RTX_REF_PRIM(RTX_PRIM_SPHERE, fs.spheres.size());
                fs.spheres.push_back(sp);
                refs[h] = r;
            } else if (auto q = dynamic_cast<const Quad*>(h)) {  // hittables.go:138-165
                rtx_quad qd{};
                qd.q[0] = q->Q.X; qd.q[1] = q->Q.Y; qd.q[2] = q->Q.Z;
                qd.u[0] = q->u.X; qd.u[1] = q->u.Y; qd.u[2] = q->u.Z;
                qd.v[0] = q->v.X; qd.v[1] = q->v.Y; qd.v[2] = q->v.Z;
                qd.w[0] = q->w.X; qd.w[1] = q->w.Y; qd.w[2] = q->w.Z;
                qd.normal[0] = q->normal.X; qd.normal[1] = q->normal.Y; qd.normal[2] = q->normal.Z;
                qd.d = q->D;
                if (!material(q->material, qd.material)) return false;
                r = RTX_REF_PRIM(RTX_PRIM_QUAD, fs.quads.size());
                fs.quads.push_back(qd);
                refs[h] = r;
            } else if (auto w = dynamic_cast<const World*>(h)) {  // a nested World: a list ref (ABI 5)
                // (an empty World is a miss, hittables.go:55-72: a list of no items, which emits nothing)
                rtx_list l{(uint32_t)fs.list_refs.size(), (uint32_t)w->hittables.size()};
                r = RTX_REF_PRIM(RTX_PRIM_LIST, fs.lists.size());
                fs.lists.push_back(l);
                fs.list_refs.resize(fs.list_refs.size() + l.count, 0);
                refs[h] = r;
                for (uint32_t k = l.count; k-- > 0;)
                    stack.push_back({w->hittables[k].get(), Patch{(int32_t)(l.first + k), 2, nullptr}});
            } else {
                return fail(RTX_ERR_UNSUPPORTED, "unknown Hittable type");
            }
            if (patch.side < 0) *patch.ext = r;
            else if (patch.side == 0) fs.nodes[patch.node].left = r;
            else if (patch.side == 1) fs.nodes[patch.node].right = r;
            else fs.list_refs[(size_t)patch.node] = r;
        }
        return true;
    }
};

}  // namespace

Error Flatten(const HittablePtr& world, FlatScene& fs) {
    fs = FlatScene{};
    if (!world) return Error{RTX_ERR_INVALID_ARG, "nil world"};
    Flattener f(fs);
    if (auto w = dynamic_cast<const World*>(world.get())) {
        for (const auto& h : w->hittables) {
            int32_t r = 0;
            if (!f.ref(h, r)) return f.err;
            fs.roots.push_back(r);
        }
        if (fs.roots.empty()) return Error{RTX_ERR_INVALID_ARG, "empty World"};
    } else {
        int32_t r = 0;
        if (!f.ref(world, r)) return f.err;
        fs.roots.push_back(r);
    }
    fs.mat_index = f.mats;
    rtx_scene_desc& d = fs.desc;
    d = rtx_scene_desc{};
    d.nodes = fs.nodes.data();
    d.n_nodes = (uint32_t)fs.nodes.size();
    d.roots = fs.roots.data();
    d.n_roots = (uint32_t)fs.roots.size();
    d.spheres = fs.spheres.data();
    d.n_spheres = (uint32_t)fs.spheres.size();
    d.quads = fs.quads.data();
    d.n_quads = (uint32_t)fs.quads.size();
    d.materials = fs.materials.data();
    d.n_materials = (uint32_t)fs.materials.size();
    d.textures = fs.textures.data();
    d.n_textures = (uint32_t)fs.textures.size();
    d.texels = fs.texels.data();
    d.n_texels = fs.texels.size();
    d.lists = fs.lists.data();
    d.n_lists = (uint32_t)fs.lists.size();
    d.list_refs = fs.list_refs.data();
    d.n_list_refs = (uint32_t)fs.list_refs.size();
    return Error{};
}

}  // namespace internal
