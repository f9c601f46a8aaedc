/* sbvh_model.c -- spatial-split Bvh2 for the traversal model (analysis tool).
 *
 * Builds a binary tree with single-triangle leaves (the Bvh2 record shape the product traverses)
 * by binned SAH over the three axes, optionally with spatial splits (Stich et al. 2009; the
 * reference's RadeonRays has them as SplitBvh, third_party/RadeonRays/RadeonRays/src/accelerator/
 * split_bvh.cpp, behind "bvh.sah.use_splits", which its Bvh2/LDS intersector does not read:
 * intersector_lds.cpp builds a plain Bvh2).  Output nodes are in tools/trav_sim.c's format, so
 * the same rays can be replayed over the reference tree and this one.
 *
 *   int sbvh_build(const Node* leaves, int ntri, Node* out, int max_out,
 *                  float alpha, int max_split_depth, float budget)
 *     leaves: the scene's triangle leaves (lmin/lmax/rmin = v0/v1/v2, mesh, prim)
 *     alpha:  spatial splits are tried when the best object split's child boxes overlap by more
 *             than alpha x the root's surface area (alpha < 0: never)
 *     budget: at most budget x ntri extra references
 *   returns the node count (root at 0), or -1 when out is too small.
 * Build: gcc -O2 -shared -fPIC tools/sbvh_model.c -o /tmp/sbvh_model.so -lm
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float lmin[3]; uint32_t left; float lmax[3]; uint32_t mesh; float rmin[3]; uint32_t right; float rmax[3]; uint32_t prim; } Node;
typedef struct { float lo[3], hi[3]; } Box;
typedef struct { Box b; int tri; } Ref;
#define INV 0xffffffffu
#define NB 32

static const Node* g_tri;
static Node* g_out;
static int g_n, g_max;
static long g_extra, g_budget;
static float g_alpha_area;
static int g_max_depth;

static Box empty_box(void) {
    Box b;
    for (int k = 0; k < 3; ++k) { b.lo[k] = FLT_MAX; b.hi[k] = -FLT_MAX; }
    return b;
}
static void grow(Box* a, const Box* b) {
    for (int k = 0; k < 3; ++k) { a->lo[k] = fminf(a->lo[k], b->lo[k]); a->hi[k] = fmaxf(a->hi[k], b->hi[k]); }
}
static void grow_pt(Box* a, const float* p) {
    for (int k = 0; k < 3; ++k) { a->lo[k] = fminf(a->lo[k], p[k]); a->hi[k] = fmaxf(a->hi[k], p[k]); }
}
static float area(const Box* b) {
    float d0 = b->hi[0] - b->lo[0], d1 = b->hi[1] - b->lo[1], d2 = b->hi[2] - b->lo[2];
    if (d0 < 0 || d1 < 0 || d2 < 0) return 0.0f;
    return 2.0f * (d0 * d1 + d1 * d2 + d0 * d2);
}
static Box isect(const Box* a, const Box* b) {
    Box r;
    for (int k = 0; k < 3; ++k) { r.lo[k] = fmaxf(a->lo[k], b->lo[k]); r.hi[k] = fminf(a->hi[k], b->hi[k]); }
    return r;
}
static void tri_verts(int t, float v[3][3]) {
    const Node* n = &g_tri[t];
    for (int k = 0; k < 3; ++k) { v[0][k] = n->lmin[k]; v[1][k] = n->lmax[k]; v[2][k] = n->rmin[k]; }
}
/* bounds of the part of triangle t inside lo <= x[axis] <= hi, intersected with the reference box */
static Box clip_tri(int t, int axis, float lo, float hi, const Box* rb) {
    float v[3][3];
    tri_verts(t, v);
    Box b = empty_box();
    for (int e = 0; e < 3; ++e) {
        const float* p = v[e];
        const float* q = v[(e + 1) % 3];
        if (p[axis] >= lo && p[axis] <= hi) grow_pt(&b, p);
        const float planes[2] = {lo, hi};
        for (int s = 0; s < 2; ++s) {
            const float c = planes[s];
            if ((p[axis] < c && q[axis] > c) || (p[axis] > c && q[axis] < c)) {
                const float f = (c - p[axis]) / (q[axis] - p[axis]);
                float x[3];
                for (int k = 0; k < 3; ++k) x[k] = p[k] + f * (q[k] - p[k]);
                x[axis] = c;
                grow_pt(&b, x);
            }
        }
    }
    return isect(&b, rb);
}

static int new_node(void) {
    if (g_n >= g_max) return -1;
    memset(&g_out[g_n], 0, sizeof(Node));
    return g_n++;
}

typedef struct { float cost; int axis; int kind; float pos; int bin; Box l, r; int nl, nr; } Split;

static void object_split(const Ref* refs, int n, Split* best) {
    Box cb = empty_box();
    for (int i = 0; i < n; ++i) {
        float c[3];
        for (int k = 0; k < 3; ++k) c[k] = 0.5f * (refs[i].b.lo[k] + refs[i].b.hi[k]);
        grow_pt(&cb, c);
    }
    for (int a = 0; a < 3; ++a) {
        const float ext = cb.hi[a] - cb.lo[a];
        if (!(ext > 0.0f)) continue;
        Box bb[NB];
        int cnt[NB] = {0};
        for (int i = 0; i < NB; ++i) bb[i] = empty_box();
        const float sc = NB / ext;
        for (int i = 0; i < n; ++i) {
            const float c = 0.5f * (refs[i].b.lo[a] + refs[i].b.hi[a]);
            int k = (int)((c - cb.lo[a]) * sc);
            k = k < 0 ? 0 : (k >= NB ? NB - 1 : k);
            grow(&bb[k], &refs[i].b);
            cnt[k]++;
        }
        Box rb[NB];
        int rc[NB];
        Box acc = empty_box();
        int ac = 0;
        for (int i = NB - 1; i > 0; --i) { grow(&acc, &bb[i]); ac += cnt[i]; rb[i] = acc; rc[i] = ac; }
        acc = empty_box();
        ac = 0;
        for (int i = 0; i < NB - 1; ++i) {
            grow(&acc, &bb[i]);
            ac += cnt[i];
            if (ac == 0 || rc[i + 1] == 0) continue;
            const float cost = area(&acc) * ac + area(&rb[i + 1]) * rc[i + 1];
            if (cost < best->cost) {
                best->cost = cost; best->axis = a; best->kind = 0; best->bin = i;
                best->pos = cb.lo[a] + (i + 1) / sc;   /* centroid bin boundary */
                best->l = acc; best->r = rb[i + 1]; best->nl = ac; best->nr = rc[i + 1];
            }
        }
    }
}

static void spatial_split(const Ref* refs, int n, const Box* nb, Split* best) {
    for (int a = 0; a < 3; ++a) {
        const float lo = nb->lo[a], ext = nb->hi[a] - nb->lo[a];
        if (!(ext > 0.0f)) continue;
        Box bb[NB];
        int ent[NB] = {0}, ex[NB] = {0};
        for (int i = 0; i < NB; ++i) bb[i] = empty_box();
        const float w = ext / NB;
        for (int i = 0; i < n; ++i) {
            int b0 = (int)((refs[i].b.lo[a] - lo) / w), b1 = (int)((refs[i].b.hi[a] - lo) / w);
            b0 = b0 < 0 ? 0 : (b0 >= NB ? NB - 1 : b0);
            b1 = b1 < 0 ? 0 : (b1 >= NB ? NB - 1 : b1);
            if (b1 < b0) b1 = b0;
            if (b0 == b1) {
                grow(&bb[b0], &refs[i].b);
            } else {
                for (int k = b0; k <= b1; ++k) {
                    const Box c = clip_tri(refs[i].tri, a, lo + k * w, k == NB - 1 ? nb->hi[a] : lo + (k + 1) * w, &refs[i].b);
                    if (c.lo[0] <= c.hi[0]) grow(&bb[k], &c);
                }
            }
            ent[b0]++;
            ex[b1]++;
        }
        Box rb[NB];
        int rc[NB];
        Box acc = empty_box();
        int ac = 0;
        for (int i = NB - 1; i > 0; --i) { grow(&acc, &bb[i]); ac += ex[i]; rb[i] = acc; rc[i] = ac; }
        acc = empty_box();
        ac = 0;
        for (int i = 0; i < NB - 1; ++i) {
            grow(&acc, &bb[i]);
            ac += ent[i];
            if (ac == 0 || rc[i + 1] == 0 || ac >= n || rc[i + 1] >= n) continue;
            const float cost = area(&acc) * ac + area(&rb[i + 1]) * rc[i + 1];
            if (cost < best->cost) {
                best->cost = cost; best->axis = a; best->kind = 1; best->bin = i;
                best->pos = lo + (i + 1) * w;
                best->l = acc; best->r = rb[i + 1]; best->nl = ac; best->nr = rc[i + 1];
            }
        }
    }
}

static void make_leaf(int idx, int tri) {
    const Node* t = &g_tri[tri];
    Node* o = &g_out[idx];
    *o = *t;
    o->left = INV;
    o->right = INV;
}

/* builds the subtree of refs[0..n) into node idx; box = the refs' bounds; takes ownership of refs */
static int build(Ref* refs, int n, int idx, const Box* box, int depth) {
    if (n == 1) {
        make_leaf(idx, refs[0].tri);
        free(refs);
        return 0;
    }
    Split s;
    s.cost = FLT_MAX;
    s.kind = -1;
    object_split(refs, n, &s);
    if (g_alpha_area >= 0.0f && depth < g_max_depth && g_extra + n <= g_budget) {   /* worst case: all split */
        const float ov = s.kind == 0 ? area((Box[]){isect(&s.l, &s.r)}) : FLT_MAX;
        if (ov > g_alpha_area) spatial_split(refs, n, box, &s);
    }
    Ref* L = (Ref*)malloc(sizeof(Ref) * (size_t)n * 2);
    Ref* R = (Ref*)malloc(sizeof(Ref) * (size_t)n * 2);
    int nl = 0, nr = 0;
    Box lb = empty_box(), rbx = empty_box();
    if (s.kind == 0) {
        for (int i = 0; i < n; ++i) {
            const float c = 0.5f * (refs[i].b.lo[s.axis] + refs[i].b.hi[s.axis]);
            if (c < s.pos) { L[nl++] = refs[i]; grow(&lb, &refs[i].b); } else { R[nr++] = refs[i]; grow(&rbx, &refs[i].b); }
        }
    } else if (s.kind == 1) {
        const float AL = area(&s.l), AR = area(&s.r);
        for (int i = 0; i < n; ++i) {
            const Ref* r = &refs[i];
            if (r->b.hi[s.axis] <= s.pos) { L[nl++] = *r; grow(&lb, &r->b); continue; }
            if (r->b.lo[s.axis] >= s.pos) { R[nr++] = *r; grow(&rbx, &r->b); continue; }
            /* straddling: split, or keep whole on one side (reference unsplitting) */
            Box l1 = s.l, r1 = s.r;
            grow(&l1, &r->b);
            grow(&r1, &r->b);
            const float cs = AL * s.nl + AR * s.nr;
            const float c1 = area(&l1) * s.nl + AR * (s.nr - 1);
            const float c2 = AL * (s.nl - 1) + area(&r1) * s.nr;
            if (c1 < cs && c1 <= c2) { L[nl++] = *r; grow(&lb, &r->b); continue; }
            if (c2 < cs) { R[nr++] = *r; grow(&rbx, &r->b); continue; }
            Ref a = *r, b = *r;
            Box big = *box;
            a.b = clip_tri(r->tri, s.axis, big.lo[s.axis], s.pos, &r->b);
            b.b = clip_tri(r->tri, s.axis, s.pos, big.hi[s.axis], &r->b);
            L[nl++] = a; grow(&lb, &a.b);
            R[nr++] = b; grow(&rbx, &b.b);
            g_extra++;
        }
    }
    if (s.kind < 0 || nl == 0 || nr == 0 || nl >= n + n || nr >= n + n || (s.kind == 1 && (nl >= n && nr >= n))) {
        /* no usable split (coincident centroids): halves in array order */
        nl = n / 2;
        nr = n - nl;
        lb = empty_box();
        rbx = empty_box();
        for (int i = 0; i < nl; ++i) { L[i] = refs[i]; grow(&lb, &refs[i].b); }
        for (int i = 0; i < nr; ++i) { R[i] = refs[nl + i]; grow(&rbx, &refs[nl + i].b); }
    }
    free(refs);
    const int li = new_node(), ri = new_node();
    if (li < 0 || ri < 0) { free(L); free(R); return -1; }
    Node* o = &g_out[idx];
    memcpy(o->lmin, lb.lo, 12); memcpy(o->lmax, lb.hi, 12);
    memcpy(o->rmin, rbx.lo, 12); memcpy(o->rmax, rbx.hi, 12);
    o->left = (uint32_t)li;
    o->right = (uint32_t)ri;
    if (build(L, nl, li, &lb, depth + 1) < 0) { free(R); return -1; }
    return build(R, nr, ri, &rbx, depth + 1);
}

int sbvh_build(const Node* leaves, int ntri, Node* out, int max_out, float alpha, int max_split_depth, float budget) {
    g_tri = leaves;
    g_out = out;
    g_max = max_out;
    g_n = 0;
    g_extra = 0;
    g_budget = (long)(budget * ntri);
    g_max_depth = max_split_depth;
    Ref* refs = (Ref*)malloc(sizeof(Ref) * (size_t)ntri);
    Box root = empty_box();
    for (int i = 0; i < ntri; ++i) {
        float v[3][3];
        tri_verts(i, v);
        Box b = empty_box();
        for (int k = 0; k < 3; ++k) grow_pt(&b, v[k]);
        refs[i].b = b;
        refs[i].tri = i;
        grow(&root, &b);
    }
    g_alpha_area = alpha < 0.0f ? -1.0f : alpha * area(&root);
    const int r = new_node();
    if (r < 0) return -1;
    if (build(refs, ntri, r, &root, 0) < 0) return -1;
    return g_n;
}

long sbvh_extra_refs(void) { return g_extra; }
