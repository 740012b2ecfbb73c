// rvcp_bvh.cpp -- host-side builder of the opt-in BVH (rvcp_config_t.accel = RVCP_ACCEL_BVH).
//
// Binary tree, binned SAH (16 bins on centroids, along the widest centroid axis) down to
// kBvhLeafMax triangles; below depth kSahDepth (or when SAH finds no useful split) the node is
// split at the centroid median; the SAH depth is capped so that SAH levels + median levels
// (ceil(log2(n / leaf)) + 1) stay below the device traversal stack (kBvhStack).  Triangles are stored in leaf order
// (TriRecord copies) together with their original face index, which the device uses for the
// scan's tie rule and the hit record.
//
// Box enlargement: every child box grows by 1e-5 of the scene diagonal plus 1e-6 of its own
// largest coordinate magnitude.  An exact triangle test (tri_accept) that accepts a hit on a
// well-conditioned ray (not nearly parallel to the triangle plane) puts the hit point within a
// few ulps of the triangle, far inside that margin, so culling never drops a hit the
// brute-force scan would find (DESIGN.md §4.6 for the nearly-parallel exception).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/rvcp.h"
#include "rvcp_internal.h"

namespace rvcp {

namespace {

struct Box {
    float lo[3] = {INFINITY, INFINITY, INFINITY};
    float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const float *p) {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], p[k]);
            hi[k] = std::max(hi[k], p[k]);
        }
    }
    void grow(const Box &b) {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    float area() const {
        if (!(hi[0] >= lo[0])) return 0.0f;
        const float x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
        return 2.0f * (x * y + y * z + z * x);
    }
};

struct Prim {
    Box box;
    float c[3];
    uint32_t id;
};

constexpr int kBins = 16;
constexpr int kSahDepthMax = 16;

struct Builder {
    std::vector<Prim> prims;
    std::vector<BvhNode> nodes;
    std::vector<uint32_t> order;
    float pad_abs = 0.0f;
    int max_depth = 0;
    int sah_depth = kSahDepthMax;

    void store_box(float *dst, const Box &b) const {
        for (int k = 0; k < 3; k++) {
            const float mag = std::max(std::fabs(b.lo[k]), std::fabs(b.hi[k]));
            const float pad = pad_abs + 1e-6f * mag;
            dst[k] = b.lo[k] - pad;
            dst[3 + k] = b.hi[k] + pad;
        }
    }

    int32_t leaf(uint32_t first, uint32_t count) {
        // leaves start at even slots: the packed 10-float leaf records (rvcp_host.cpp) are then
        // 16-B aligned; the padding slot holds kBvhPadId and is never inside a leaf's range
        if (order.size() & 1u) order.push_back(kBvhPadId);
        const uint32_t start = (uint32_t)order.size();
        for (uint32_t i = first; i < first + count; i++) order.push_back(prims[i].id);
        return ~(int32_t)((start << 5) | (count - 1));
    }

    // Build [first, first + count) and return its reference.
    int32_t build(uint32_t first, uint32_t count, int depth, Box *out_box) {
        Box bounds, cbounds;
        for (uint32_t i = first; i < first + count; i++) {
            bounds.grow(prims[i].box);
            cbounds.grow(prims[i].c);
        }
        *out_box = bounds;
        max_depth = std::max(max_depth, depth);
        if (count <= (uint32_t)kBvhLeafMax) return leaf(first, count);

        int axis = 0;
        for (int k = 1; k < 3; k++)
            if (cbounds.hi[k] - cbounds.lo[k] > cbounds.hi[axis] - cbounds.lo[axis]) axis = k;
        const float ext = cbounds.hi[axis] - cbounds.lo[axis];
        uint32_t mid = first + count / 2;
        bool sah_ok = false;
        if (depth < sah_depth && ext > 0.0f) {
            Box bb[kBins];
            uint32_t bn[kBins] = {};
            auto bin_of = [&](const Prim &p) {
                int b = (int)((p.c[axis] - cbounds.lo[axis]) / ext * kBins);
                return std::min(std::max(b, 0), kBins - 1);
            };
            for (uint32_t i = first; i < first + count; i++) {
                const int b = bin_of(prims[i]);
                bb[b].grow(prims[i].box);
                bn[b]++;
            }
            float best = INFINITY;
            int best_split = -1;
            for (int s = 1; s < kBins; s++) {
                Box l, r;
                uint32_t nl = 0, nr = 0;
                for (int b = 0; b < s; b++) { if (bn[b]) l.grow(bb[b]); nl += bn[b]; }
                for (int b = s; b < kBins; b++) { if (bn[b]) r.grow(bb[b]); nr += bn[b]; }
                if (!nl || !nr) continue;
                const float cost = l.area() * nl + r.area() * nr;
                if (cost < best) { best = cost; best_split = s; }
            }
            if (best_split > 0 && best < bounds.area() * count) {
                auto it = std::partition(prims.begin() + first, prims.begin() + first + count,
                                         [&](const Prim &p) { return bin_of(p) < best_split; });
                mid = (uint32_t)(it - prims.begin());
                sah_ok = mid > first && mid < first + count;
            }
        }
        if (!sah_ok) {
            std::nth_element(prims.begin() + first, prims.begin() + first + count / 2,
                             prims.begin() + first + count,
                             [&](const Prim &a, const Prim &b) {
                                 return a.c[axis] < b.c[axis] || (a.c[axis] == b.c[axis] && a.id < b.id);
                             });
            mid = first + count / 2;
        }
        const uint32_t self = (uint32_t)nodes.size();
        nodes.emplace_back();
        Box lb, rb;
        const int32_t l = build(first, mid - first, depth + 1, &lb);
        const int32_t r = build(mid, first + count - mid, depth + 1, &rb);
        BvhNode &N = nodes[self];
        store_box(N.lbox, lb);
        store_box(N.rbox, rb);
        N.left = l;
        N.right = r;
        N.pad[0] = N.pad[1] = 0;
        return (int32_t)self;
    }
};

// Early split clipping (Ernst & Greiner): a triangle much larger than the scene's typical one
// -- the Cornell walls among the C5 mesh's 100 000 small triangles -- enters the build as several
// prims, the pieces of the triangle cut at the midpoints of their longest axis until each piece
// spans at most `thr`, each with the box of its clipped polygon (clipped in double, the box
// rounded outward to float) and the triangle's own id.  The pieces' boxes cover the triangle, so
// every leaf holding a piece holds the triangle, and a ray through the triangle enters some
// piece's box; a leaf may repeat a triangle another leaf holds, and a repeated test never
// changes the hit (equal t and equal face fail the order rule).  Big boxes no longer span the
// tree's upper levels: on the C5 mesh the CPU model (tools/bvh4_check.cpp) steps 38.6 -> 35.3
// per path ray and 49.2 -> 46.7 per shadow ray for 1.6 % more prims.
// thr = max(8 x the median prim extent, scene diagonal / 16); at most n / 8 extra prims.
void early_split_clip(std::vector<Prim> &prims, const float (*pos)[3][3], const Box &scene)
{
    const size_t n = prims.size();
    if (n < 64) return;
    std::vector<float> ext(n);
    for (size_t i = 0; i < n; i++) {
        float e = 0.0f;
        for (int k = 0; k < 3; k++) e = std::max(e, prims[i].box.hi[k] - prims[i].box.lo[k]);
        ext[i] = e;
    }
    std::vector<float> sorted(ext);
    std::nth_element(sorted.begin(), sorted.begin() + n / 2, sorted.end());
    const float dx = scene.hi[0] - scene.lo[0], dy = scene.hi[1] - scene.lo[1],
                dz = scene.hi[2] - scene.lo[2];
    const float thr = std::max(8.0f * sorted[n / 2], std::sqrt(dx * dx + dy * dy + dz * dz) / 16.0f);
    if (!(thr > 0.0f) || !std::isfinite(thr)) return;
    const size_t budget = n / 8;
    std::vector<Prim> out;
    struct P3 { double x[3]; };
    struct Piece { std::vector<P3> poly; int depth; };
    for (size_t i = 0; i < n; i++) {
        if (!(ext[i] > thr) || out.size() >= budget) continue;
        const Prim src = prims[i];
        std::vector<Prim> pieces;
        std::vector<Piece> todo(1);
        for (int v = 0; v < 3; v++) {
            P3 q;
            for (int k = 0; k < 3; k++) q.x[k] = pos[src.id][v][k];
            todo[0].poly.push_back(q);
        }
        todo[0].depth = 0;
        while (!todo.empty()) {
            Piece pc = std::move(todo.back());
            todo.pop_back();
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (const P3 &q : pc.poly)
                for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], q.x[k]); hi[k] = std::max(hi[k], q.x[k]); }
            int ax = 0;
            for (int k = 1; k < 3; k++)
                if (hi[k] - lo[k] > hi[ax] - lo[ax]) ax = k;
            if (hi[ax] - lo[ax] <= thr || pc.depth >= 10) {
                Prim f;
                for (int k = 0; k < 3; k++) {
                    // outward: the float box contains the double one
                    f.box.lo[k] = std::nextafter((float)lo[k], -INFINITY);
                    f.box.hi[k] = std::nextafter((float)hi[k], INFINITY);
                    f.c[k] = 0.5f * (f.box.lo[k] + f.box.hi[k]);
                }
                f.id = src.id;
                pieces.push_back(f);
                continue;
            }
            const double m = 0.5 * (lo[ax] + hi[ax]);
            Piece L, R;
            L.depth = R.depth = pc.depth + 1;
            const size_t np = pc.poly.size();
            for (size_t j = 0; j < np; j++) {      // Sutherland-Hodgman against x_ax <= m / >= m
                const P3 &A = pc.poly[j], &Bq = pc.poly[(j + 1) % np];
                if (A.x[ax] <= m) L.poly.push_back(A);
                if (A.x[ax] >= m) R.poly.push_back(A);
                if ((A.x[ax] < m && Bq.x[ax] > m) || (A.x[ax] > m && Bq.x[ax] < m)) {
                    const double t = (m - A.x[ax]) / (Bq.x[ax] - A.x[ax]);
                    P3 C;
                    for (int k = 0; k < 3; k++) C.x[k] = A.x[k] + t * (Bq.x[k] - A.x[k]);
                    C.x[ax] = m;
                    L.poly.push_back(C);
                    R.poly.push_back(C);
                }
            }
            if (!L.poly.empty()) todo.push_back(std::move(L));
            if (!R.poly.empty()) todo.push_back(std::move(R));
        }
        if (pieces.size() <= 1) continue;
        prims[i] = pieces[0];
        out.insert(out.end(), pieces.begin() + 1, pieces.end());
    }
    prims.insert(prims.end(), out.begin(), out.end());
}

}  // namespace

uint32_t bvh_big_prefix(const float (*pos)[3][3], uint32_t n, uint32_t cap)
{
    if (n < 64) return 0;
    std::vector<float> ext(n);
    Box scene;
    for (uint32_t i = 0; i < n; i++) {
        Box b;
        bool finite = true;
        for (int v = 0; v < 3; v++)
            for (int k = 0; k < 3; k++) finite = finite && std::isfinite(pos[i][v][k]);
        if (!finite) return 0;
        for (int v = 0; v < 3; v++) b.grow(pos[i][v]);
        float e = 0.0f;
        for (int k = 0; k < 3; k++) e = std::max(e, b.hi[k] - b.lo[k]);
        ext[i] = e;
        scene.grow(b);
    }
    std::vector<float> sorted(ext);
    std::nth_element(sorted.begin(), sorted.begin() + n / 2, sorted.end());
    const float dx = scene.hi[0] - scene.lo[0], dy = scene.hi[1] - scene.lo[1],
                dz = scene.hi[2] - scene.lo[2];
    const float thr = std::max(8.0f * sorted[n / 2], std::sqrt(dx * dx + dy * dy + dz * dz) / 16.0f);
    uint32_t k = 0;
    while (k < n && k < cap && ext[k] > thr) k++;
    return k;
}

// Build over `n` faces given their three vertex positions.  Outputs the node array, the
// leaf-ordered original face ids and the root reference; returns the tree depth.
int bvh_build(const float (*pos)[3][3], uint32_t n, std::vector<BvhNode> &nodes,
              std::vector<uint32_t> &order, int32_t &root)
{
    Builder B;
    B.prims.resize(n);
    Box scene;
    for (uint32_t i = 0; i < n; i++) {
        Prim &p = B.prims[i];
        bool finite = true;
        for (int v = 0; v < 3; v++)
            for (int k = 0; k < 3; k++) finite = finite && std::isfinite(pos[i][v][k]);
        if (finite) {
            for (int v = 0; v < 3; v++) p.box.grow(pos[i][v]);
        } else {            // never accepted by the exact test (NaN/inf arithmetic): park it
            const float z[3] = {0.0f, 0.0f, 0.0f};
            p.box.grow(z);
        }
        for (int k = 0; k < 3; k++) p.c[k] = 0.5f * (p.box.lo[k] + p.box.hi[k]);
        p.id = i;
        scene.grow(p.box);
    }
    if (n == 0) {
        nodes.clear();
        order.clear();
        root = 0;
        return 0;
    }
#ifndef RVCP_BVH_NO_SPLIT_CLIP
    early_split_clip(B.prims, pos, scene);
#endif
    const float dx = scene.hi[0] - scene.lo[0], dy = scene.hi[1] - scene.lo[1],
                dz = scene.hi[2] - scene.lo[2];
    B.pad_abs = 1e-5f * std::sqrt(dx * dx + dy * dy + dz * dz);
    const uint32_t np = (uint32_t)B.prims.size();     // n plus the split-clip pieces
    int median_levels = 1;
    for (uint64_t leaves = ((uint64_t)np + kBvhLeafMax - 1) / kBvhLeafMax; leaves > 1; leaves = (leaves + 1) / 2)
        median_levels++;
    B.sah_depth = std::max(0, std::min(kSahDepthMax, kBvhStack - 1 - median_levels));
    B.nodes.reserve(2 * (size_t)np / kBvhLeafMax + 2);
    B.order.reserve(np);
    Box rootbox;
    root = B.build(0, np, 0, &rootbox);
    nodes.swap(B.nodes);
    order.swap(B.order);
    return B.max_depth;     // the caller rejects max_depth >= kBvhStack
}

namespace {

struct Collapser {
    const std::vector<BvhNode> &n2;
    std::vector<Bvh4Node> &out;
    std::vector<int> height;        // binary height per node (a leaf child counts 0)

    struct Child {
        int32_t ref;
        const float *box;           // lo xyz, hi xyz (already enlarged)
    };

    int h(int32_t ref) const { return ref < 0 ? 0 : height[ref]; }

    int measure(int32_t ref) {
        if (ref < 0) return 0;
        const int a = measure(n2[ref].left), b = measure(n2[ref].right);
        return height[ref] = 1 + std::max(a, b);
    }

    static float area(const float *b) {
        const float x = b[3] - b[0], y = b[4] - b[1], z = b[5] - b[2];
        return x * y + y * z + z * x;
    }

    // 4-wide node for binary node `ref`, whose traversal may use `budget` stack entries.
    // Children are opened (largest box first) while (children - 1) plus the largest binary
    // height among them fits the budget; an unopened binary subtree of height H never needs
    // more than H entries, so every recursion stays feasible.
    int32_t build(int32_t ref, int budget, int &need) {
        const BvhNode &N = n2[ref];
        std::vector<Child> c = {{N.left, N.lbox}, {N.right, N.rbox}};
        while (c.size() < 4) {
            int pick = -1;
            float best = -1.0f;
            for (size_t i = 0; i < c.size(); i++)
                if (c[i].ref >= 0 && area(c[i].box) > best) { best = area(c[i].box); pick = (int)i; }
            if (pick < 0) break;
            const BvhNode &M = n2[c[pick].ref];
            std::vector<Child> t = c;
            t[pick] = {M.left, M.lbox};
            t.push_back({M.right, M.rbox});
            int hmax = 0;
            for (const Child &x : t) hmax = std::max(hmax, h(x.ref));
            if ((int)t.size() - 1 + hmax > budget) break;
            c.swap(t);
        }
        const int32_t self = (int32_t)out.size();
        out.emplace_back();
        const int push = (int)c.size() - 1;
        int sub = 0;
        int32_t refs[4];
        for (size_t i = 0; i < c.size(); i++) {
            refs[i] = c[i].ref;
            if (c[i].ref >= 0) {
                int nd = 0;
                refs[i] = build(c[i].ref, budget - push, nd);
                sub = std::max(sub, nd);
            }
        }
        Bvh4Node &Q = out[self];
        for (int i = 0; i < 4; i++) {
            const bool used = i < (int)c.size();
            for (int k = 0; k < 3; k++) {
                Q.lo[k][i] = used ? c[i].box[k] : 3e38f;
                Q.hi[k][i] = used ? c[i].box[3 + k] : 3e38f;
            }
            Q.ref[i] = used ? refs[i] : ~0;
            Q.pad[i] = 0;
        }
        need = push + sub;
        return self;
    }
};

}  // namespace

int bvh4_collapse(const std::vector<BvhNode> &nodes, int32_t root, std::vector<Bvh4Node> &out,
                  int32_t &root4)
{
    out.clear();
    if (root < 0) {             // a single leaf: no inner node
        root4 = root;
        return 0;
    }
    Collapser C{nodes, out, std::vector<int>(nodes.size(), 0)};
    C.measure(root);
    out.reserve(nodes.size());
    int need = 0;
    root4 = C.build(root, kBvhStack, need);
    return need;
}

// Byte quantisation of the 4-wide nodes (Bvh4QNode).  Per node and axis: origin = the
// smallest child lo (a float), scale = the smallest power of two (>= 2^-60) with
// (largest child hi - origin) / scale <= 255, q_lo = floor((lo - origin) / scale),
// q_hi = ceil((hi - origin) / scale), evaluated in double, where both are exact (scale is a
// power of two and the operands floats).  So origin + q_lo * scale <= lo and
// origin + q_hi * scale >= hi in exact arithmetic: every quantised box contains its float box,
// which already carries the build's enlargement (far above the few-ulp rounding of the
// kernel's decode), so the traversal culls nothing the float boxes keep.
void bvh4_quantize(const std::vector<Bvh4Node> &in, std::vector<Bvh4QNode> &out)
{
    out.resize(in.size());
    for (size_t j = 0; j < in.size(); j++) {
        const Bvh4Node &N = in[j];
        Bvh4QNode &Q = out[j];
        for (int k = 0; k < 3; k++) {
            float lo = 0.0f, hi = 0.0f;
            bool any = false;
            for (int c = 0; c < 4; c++) {
                if (N.ref[c] == ~0) continue;
                lo = any ? std::min(lo, N.lo[k][c]) : N.lo[k][c];
                hi = any ? std::max(hi, N.hi[k][c]) : N.hi[k][c];
                any = true;
            }
            const double ext = any ? (double)hi - (double)lo : 0.0;
            int e = -60;
            while (std::ldexp(255.0, e) < ext) e++;
            const double sc = std::ldexp(1.0, e);
            Q.origin[k] = lo;
            Q.scale[k] = (float)sc;
            uint32_t wl = 0, wh = 0;
            for (int c = 0; c < 4; c++) {
                uint32_t ql = 255, qh = 0;                     // unused: inverted, never entered
                if (N.ref[c] != ~0) {
                    ql = (uint32_t)std::floor(((double)N.lo[k][c] - (double)lo) / sc);
                    qh = (uint32_t)std::ceil(((double)N.hi[k][c] - (double)lo) / sc);
                    if (qh > 255) qh = 255;                    // cannot happen: ext / sc <= 255
                }
                wl |= ql << (8 * c);
                wh |= qh << (8 * c);
            }
            Q.qlo[k] = wl;
            Q.qhi[k] = wh;
        }
        for (int c = 0; c < 4; c++) Q.ref[c] = N.ref[c];
    }
}

}  // namespace rvcp
