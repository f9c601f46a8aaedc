/* trav_sim.c -- CPU model of the GPU traversal's dependent-fetch structure (analysis tool).
 *
 * Replays the Bvh2 closest/any traversal (intersect_bvh2_lds.cl:66-363, same node order as
 * the oracle) and counts, per ray, the node records visited and the number of dependent
 * fetch rounds under schemes that fetch several records in one round:
 *   K = 1  one record per round (the current kernel);
 *   K = k  a round fetches the current record plus, while the records already chosen are
 *          leaves, the next stack entries (the nodes a leaf's pop will reach), up to k records.
 * A leaf never changes which node comes next (closest-hit pops after every leaf), so the
 * k-record rounds visit exactly the reference's sequence.  Waves = 64 consecutive rays;
 * a wave's rounds = the max over its lanes.
 * Build: gcc -O2 -shared -fPIC tools/trav_sim.c -o /tmp/trav_sim.so -lm
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct { float lmin[3]; uint32_t left; float lmax[3]; uint32_t mesh; float rmin[3]; uint32_t right; float rmax[3]; uint32_t prim; } Node;
typedef struct { float o[4]; float d[4]; int32_t extra[2]; int32_t bf; int32_t pad; } Ray;
#define INV 0xffffffffu
#define KMAX 4

static inline float sinv(float d) { return 1.0f / (fabsf(d) > 1e-8f ? d : copysignf(1e-8f, d)); }

static void bbox(const float* lo, const float* hi, const float* inv, const float* oxi, float tmax, float* t0, float* t1) {
    float f[3], n[3];
    for (int k = 0; k < 3; ++k) { f[k] = fmaf(hi[k], inv[k], oxi[k]); n[k] = fmaf(lo[k], inv[k], oxi[k]); }
    *t1 = fminf(fminf(fminf(fmaxf(f[0], n[0]), fmaxf(f[1], n[1])), fmaxf(f[2], n[2])), tmax);
    *t0 = fmaxf(fmaxf(fmaxf(fminf(f[0], n[0]), fminf(f[1], n[1])), fminf(f[2], n[2])), 0.f);
}
static float tri(const Ray* r, const Node* n, float tmax) {
    float e1[3], e2[3], s1[3], d[3], s2[3];
    for (int k = 0; k < 3; ++k) { e1[k] = n->lmax[k] - n->lmin[k]; e2[k] = n->rmin[k] - n->lmin[k]; }
    s1[0] = r->d[1] * e2[2] - r->d[2] * e2[1]; s1[1] = r->d[2] * e2[0] - r->d[0] * e2[2]; s1[2] = r->d[0] * e2[1] - r->d[1] * e2[0];
    float den = s1[0] * e1[0] + s1[1] * e1[1] + s1[2] * e1[2];
    if (den == 0.f) return tmax;
    float id = 1.0f / den;
    for (int k = 0; k < 3; ++k) d[k] = r->o[k] - n->lmin[k];
    float b1 = (d[0] * s1[0] + d[1] * s1[1] + d[2] * s1[2]) * id;
    s2[0] = d[1] * e1[2] - d[2] * e1[1]; s2[1] = d[2] * e1[0] - d[0] * e1[2]; s2[2] = d[0] * e1[1] - d[1] * e1[0];
    float b2 = (r->d[0] * s2[0] + r->d[1] * s2[1] + r->d[2] * s2[2]) * id;
    float t = (e2[0] * s2[0] + e2[1] * s2[1] + e2[2] * s2[2]) * id;
    if (b1 < 0.f || b1 > 1.f || b2 < 0.f || b1 + b2 > 1.f || t < 0.f || t > tmax) return tmax;
    return t;
}

/* out per ray: [0] visits, [1] leaf visits, [2..2+KMAX-1] rounds for K=1..KMAX,
 * [2+KMAX] internal visits reached by descent (not by a pop); hit_t/hit_node */
static int g_order = 0;   /* any-hit child order: 0 near first (RR), 1 far first, 2 larger box first, 3 leaf first */
void set_order(int o) { g_order = o; }
static float area(const float* lo, const float* hi) {
    float d0 = hi[0] - lo[0], d1 = hi[1] - lo[1], d2 = hi[2] - lo[2];
    return d0 * d1 + d1 * d2 + d0 * d2;
}
void sim(const Node* nodes, const Ray* rays, int n, int any, int32_t* out, float* hit_t, int32_t* hit_node) {
    static uint32_t stack[1 << 16];
    static uint32_t seq[1 << 20];
    static uint8_t leaf[1 << 20];
    static uint32_t stk_at[1 << 20]; /* stack depth when the record was chosen (for the K>1 rule) */
    (void)stk_at;
    for (int i = 0; i < n; ++i) {
        const Ray* r = &rays[i];
        int32_t* o = out + (size_t)i * (3 + KMAX);
        memset(o, 0, sizeof(int32_t) * (3 + KMAX));
        if (r->extra[1] == 0) { hit_t[i] = -1; hit_node[i] = -1; continue; }
        float inv[3], oxi[3];
        for (int k = 0; k < 3; ++k) { inv[k] = sinv(r->d[k]); oxi[k] = -r->o[k] * inv[k]; }
        float ct = r->o[3];
        uint32_t addr = 0, best = INV;
        int sp = 0, nv = 0, desc = 1, ndesc = 0;
        stack[sp++] = INV;
        /* The K>1 rule needs, at each round start, whether the chosen records are leaves: we
         * record the visit sequence and the leaf flags, then group afterwards. A round that
         * starts at visit j takes visits j..j+m-1 while visits j..j+m-2 are leaves and each
         * next visit is a POP target (true after any leaf). */
        while (addr != INV) {
            const Node* nd = &nodes[addr];
            int isleaf = nd->left == INV;
            if (nv < (1 << 20)) { seq[nv] = addr; leaf[nv] = (uint8_t)isleaf; }
            ++nv;
            if (!isleaf && desc) ++ndesc;
            if (!isleaf) {
                float a0, a1, b0, b1;
                bbox(nd->lmin, nd->lmax, inv, oxi, ct, &a0, &a1);
                bbox(nd->rmin, nd->rmax, inv, oxi, ct, &b0, &b1);
                int h0 = a0 <= a1, h1 = b0 <= b1, c1 = h1 && (a0 > b0);
                if (any && g_order == 1) c1 = h1 && !(a0 > b0);
                if (any && g_order == 2) c1 = h1 && (area(nd->rmin, nd->rmax) > area(nd->lmin, nd->lmax));
                if (any && g_order == 3) {
                    int lL = nodes[nd->left].left == INV, lR = nodes[nd->right].left == INV;
                    c1 = h1 && ((lR && !lL) || (lR == lL && a0 > b0));
                }
                if (h0 || h1) {
                    uint32_t def;
                    if (c1 || !h0) { addr = nd->right; def = nd->left; } else { addr = nd->left; def = nd->right; }
                    if (h0 && h1) stack[sp++] = def;
                    desc = 1;
                    continue;
                }
            } else if (r->extra[0] != (int)nd->mesh) {
                float t = tri(r, nd, ct);
                if (t < ct) {
                    ct = t; best = addr;
                    if (any) break;
                }
            }
            addr = stack[--sp];
            desc = 0;
        }
        o[0] = nv;
        o[2 + KMAX] = ndesc;
        int lv = 0;
        for (int j = 0; j < nv && j < (1 << 20); ++j) lv += leaf[j];
        o[1] = lv;
        for (int K = 1; K <= KMAX; ++K) {
            int rounds = 0, j = 0;
            while (j < nv) {
                int m = 1;
                while (m < K && j + m - 1 < nv && leaf[j + m - 1] && j + m < nv) ++m;
                j += m;
                ++rounds;
            }
            o[1 + K] = rounds;
        }
        hit_t[i] = ct;
        hit_node[i] = best == INV ? -1 : (int32_t)best;
    }
}

/* Leaf-pair schemes.  out per ray: [0] visits (= loop iterations now),
 * [1] iterations when an internal node whose two children are both leaves and whose two boxes
 * the ray hits tests both triangles in ONE iteration (their records fetched together, nearer
 * first; the far leaf is not pushed), [2] iterations when such a leaf-pair parent's record
 * carries both triangles (one iteration covers the parent and whichever leaves it hits),
 * [3] leaf-pair parents visited, [4] of them with both boxes hit. */
void sim_pairs(const Node* nodes, const Ray* rays, int n, int any, int32_t* out) {
    static uint32_t stack[1 << 16];
    for (int i = 0; i < n; ++i) {
        const Ray* r = &rays[i];
        int32_t* o = out + (size_t)i * 5;
        memset(o, 0, sizeof(int32_t) * 5);
        if (r->extra[1] == 0) continue;
        float inv[3], oxi[3];
        for (int k = 0; k < 3; ++k) { inv[k] = sinv(r->d[k]); oxi[k] = -r->o[k] * inv[k]; }
        float ct = r->o[3];
        uint32_t addr = 0;
        int sp = 0, nv = 0, p1 = 0, p2 = 0, pp = 0, pb = 0;
        stack[sp++] = INV;
        while (addr != INV) {
            const Node* nd = &nodes[addr];
            ++nv; ++p1; ++p2;
            if (nd->left != INV) {
                float a0, a1, b0, b1;
                bbox(nd->lmin, nd->lmax, inv, oxi, ct, &a0, &a1);
                bbox(nd->rmin, nd->rmax, inv, oxi, ct, &b0, &b1);
                int h0 = a0 <= a1, h1 = b0 <= b1, c1 = h1 && (a0 > b0);
                int pair = nodes[nd->left].left == INV && nodes[nd->right].left == INV;
                if (pair) {
                    ++pp;
                    if (h0 && h1) ++pb;
                    /* the leaves this node reaches: nearer first, each tested against the t so far */
                    uint32_t first = (c1 || !h0) ? nd->right : nd->left, second = (c1 || !h0) ? nd->left : nd->right;
                    int nl = (h0 ? 1 : 0) + (h1 ? 1 : 0);
                    int done = 0;
                    for (int k = 0; k < nl && !done; ++k) {
                        const Node* lf = &nodes[k == 0 ? first : second];
                        ++nv;
                        if (r->extra[0] != (int)lf->mesh) {
                            float t = tri(r, lf, ct);
                            if (t < ct) { ct = t; if (any) done = 1; }
                        }
                    }
                    p1 += nl ? 1 : 0;   /* both hit: one iteration for the two; one hit: its own */
                    if (done) break;
                    addr = stack[--sp];
                    continue;
                }
                if (h0 || h1) {
                    uint32_t def;
                    if (c1 || !h0) { addr = nd->right; def = nd->left; } else { addr = nd->left; def = nd->right; }
                    if (h0 && h1) stack[sp++] = def;
                    continue;
                }
            } else if (r->extra[0] != (int)nd->mesh) {
                float t = tri(r, nd, ct);
                if (t < ct) { ct = t; if (any) break; }
            }
            addr = stack[--sp];
        }
        o[0] = nv; o[1] = p1; o[2] = p2; o[3] = pp; o[4] = pb;
    }
}

/* Visits by tree level (analysis of an LDS-resident top of the tree): hist[min(level, 63)] +=
 * visits of nodes at that level (root = 0), over the closest / any traversal of n rays. */
void sim_levels(const Node* nodes, const uint8_t* level, const Ray* rays, int n, int any, int64_t* hist) {
    static uint32_t stack[1 << 16];
    for (int i = 0; i < n; ++i) {
        const Ray* r = &rays[i];
        if (r->extra[1] == 0) continue;
        float inv[3], oxi[3];
        for (int k = 0; k < 3; ++k) { inv[k] = sinv(r->d[k]); oxi[k] = -r->o[k] * inv[k]; }
        float ct = r->o[3];
        uint32_t addr = 0;
        int sp = 0;
        stack[sp++] = INV;
        while (addr != INV) {
            const Node* nd = &nodes[addr];
            hist[level[addr] < 63 ? level[addr] : 63] += 1;
            if (nd->left != INV) {
                float a0, a1, b0, b1;
                bbox(nd->lmin, nd->lmax, inv, oxi, ct, &a0, &a1);
                bbox(nd->rmin, nd->rmax, inv, oxi, ct, &b0, &b1);
                int h0 = a0 <= a1, h1 = b0 <= b1, c1 = h1 && (a0 > b0);
                if (h0 || h1) {
                    uint32_t def;
                    if (c1 || !h0) { addr = nd->right; def = nd->left; } else { addr = nd->left; def = nd->right; }
                    if (h0 && h1) stack[sp++] = def;
                    continue;
                }
            } else if (r->extra[0] != (int)nd->mesh) {
                float t = tri(r, nd, ct);
                if (t < ct) { ct = t; if (any) break; }
            }
            addr = stack[--sp];
        }
    }
}

/* Wave-packet cost model: per group of 64 consecutive rays, the number of DISTINCT nodes the
 * group's active rays (skip[i] == 0) visit in their own traversals -- a lower bound of the
 * packet walk's records (tools/shadow_cache_model.py). */
static int cmp_u32(const void* a, const void* b) {
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}
#include <stdlib.h>
void sim_union(const Node* nodes, const Ray* rays, int n, int any, const uint8_t* skip, int32_t* out_waves) {
    static uint32_t stack[1 << 16];
    uint32_t* buf = (uint32_t*)malloc(sizeof(uint32_t) * (64u << 12));
    for (int w = 0; w * 64 < n; ++w) {
        int cnt = 0;
        for (int i = w * 64; i < n && i < w * 64 + 64; ++i) {
            const Ray* r = &rays[i];
            if (r->extra[1] == 0 || skip[i]) continue;
            float inv[3], oxi[3];
            for (int k = 0; k < 3; ++k) { inv[k] = sinv(r->d[k]); oxi[k] = -r->o[k] * inv[k]; }
            float ct = r->o[3];
            uint32_t addr = 0;
            int sp = 0;
            stack[sp++] = INV;
            while (addr != INV) {
                const Node* nd = &nodes[addr];
                if (cnt < (64 << 12)) buf[cnt++] = addr;
                if (nd->left != INV) {
                    float a0, a1, b0, b1;
                    bbox(nd->lmin, nd->lmax, inv, oxi, ct, &a0, &a1);
                    bbox(nd->rmin, nd->rmax, inv, oxi, ct, &b0, &b1);
                    int h0 = a0 <= a1, h1 = b0 <= b1, c1 = h1 && (a0 > b0);
                    if (h0 || h1) {
                        uint32_t def;
                        if (c1 || !h0) { addr = nd->right; def = nd->left; } else { addr = nd->left; def = nd->right; }
                        if (h0 && h1) stack[sp++] = def;
                        continue;
                    }
                } else if (r->extra[0] != (int)nd->mesh) {
                    float t = tri(r, nd, ct);
                    if (t < ct) { ct = t; if (any) break; }
                }
                addr = stack[--sp];
            }
        }
        qsort(buf, cnt, sizeof(uint32_t), cmp_u32);
        int u = cnt ? 1 : 0;
        for (int j = 1; j < cnt; ++j) u += buf[j] != buf[j - 1];
        out_waves[w] = u;
    }
    free(buf);
}

/* Closest-hit visits when the walk starts with closest = seed[i] (a known hit distance, e.g.
 * hit_t * (1 + 1e-4)): an upper bound of what a hit-distance hint could save. out: visits. */
void sim_seeded(const Node* nodes, const Ray* rays, int n, const float* seed, int32_t* out) {
    static uint32_t stack[1 << 16];
    for (int i = 0; i < n; ++i) {
        const Ray* r = &rays[i];
        out[i] = 0;
        if (r->extra[1] == 0) continue;
        float inv[3], oxi[3];
        for (int k = 0; k < 3; ++k) { inv[k] = sinv(r->d[k]); oxi[k] = -r->o[k] * inv[k]; }
        float ct = seed[i] < r->o[3] ? seed[i] : r->o[3];
        uint32_t addr = 0;
        int sp = 0, nv = 0;
        stack[sp++] = INV;
        while (addr != INV) {
            const Node* nd = &nodes[addr];
            ++nv;
            if (nd->left != INV) {
                float a0, a1, b0, b1;
                bbox(nd->lmin, nd->lmax, inv, oxi, ct, &a0, &a1);
                bbox(nd->rmin, nd->rmax, inv, oxi, ct, &b0, &b1);
                int h0 = a0 <= a1, h1 = b0 <= b1, c1 = h1 && (a0 > b0);
                if (h0 || h1) {
                    uint32_t def;
                    if (c1 || !h0) { addr = nd->right; def = nd->left; } else { addr = nd->left; def = nd->right; }
                    if (h0 && h1) stack[sp++] = def;
                    continue;
                }
            } else if (r->extra[0] != (int)nd->mesh) {
                float t = tri(r, nd, ct);
                if (t < ct) ct = t;
            }
            addr = stack[--sp];
        }
        out[i] = nv;
    }
}
