// Host emulation of the device SAH build's algorithm (mcrt_sahbuild.hip): the closed-form
// partition (ranks instead of the two-pointer loop), the tabulated _mm_rcp_ps rule and the
// split arithmetic of mcrt_sah.h, run top-down on the CPU and compared record for record with
// the host build (mcrt_bvh.cpp, the RadeonRays Bvh2 restatement).  Exit 0 = identical.
//   usage: sah_emul [n] [seed] [kind]   kind 0 random soup, 1 grid (ties), 2 degenerate clusters
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../monte-carlo-raytracer_amd/csrc/mcrt_internal.h"
#include "../../monte-carlo-raytracer_amd/csrc/mcrt_sah.h"

using namespace mcrt;
using sah::V4;

struct Emu {
    const float* tri;
    size_t n;
    std::vector<V4> amin, amax, cen;
    std::vector<uint32_t> refs;
    std::vector<float> nodes;
    const HostRcp* R;
    uint32_t nb;
    float cost;
    bool sahOn;
    int depth = 0;

    void leaf(uint32_t node, uint32_t ref, const int32_t* shapeOf, const int32_t* primOf) {
        const float* p = &tri[9 * (size_t)ref];
        float* o = &nodes[16 * (size_t)node];
        o[0] = p[0]; o[1] = p[1]; o[2] = p[2]; std::memcpy(&o[3], &shapeOf[ref], 4);
        o[4] = p[3] - p[0]; o[5] = p[4] - p[1]; o[6] = p[5] - p[2]; std::memcpy(&o[7], &primOf[ref], 4);
        o[8] = p[6] - p[0]; o[9] = p[7] - p[1]; o[10] = p[8] - p[2]; o[11] = 0.0f;
        const int32_t m[4] = {-1, -1, 0, 0};
        std::memcpy(&o[12], m, 16);
    }
    void node(V4 bmin, V4 bmax, V4 cmin, V4 cmax, uint32_t start, uint32_t num, uint32_t index, uint32_t level,
              const int32_t* so, const int32_t* po) {
        depth = std::max(depth, (int)level);
        const uint32_t ax = sah::maxAxis(cmin, cmax);
        const float ext = sah::lane(sah::vsub(cmax, cmin), ax);
        float split = 0.5f * (sah::lane(cmax, ax) + sah::lane(cmin, ax));
        bool median = !(ext > 0.0f);
        uint32_t nL = 0;
        auto C = [&](uint32_t id) { return sah::lane(cen[id], ax); };
        if (!median) {
            if (sahOn && num > 8) {
                const float cm = sah::lane(cmin, ax);
                const float cinv = sah::rcp_ps(ext, R->t.data(), R->bits);
                const float areaInv = sah::rcp_ps(sah::sa4(bmin, bmax), R->t.data(), R->bits);
                std::vector<uint32_t> cnt(nb, 0);
                std::vector<V4> bmn(nb, V4{INFINITY, INFINITY, INFINITY, INFINITY}), bmx(nb, V4{-INFINITY, -INFINITY, -INFINITY, -INFINITY}), rmn(nb), rmx(nb);
                const uint32_t full4 = num & ~3u;
                for (uint32_t j = 0; j < num; ++j) {
                    const uint32_t id = refs[start + j];
                    const uint32_t b = j < full4 ? sah::binFull(C(id), cm, cinv, (float)nb, nb) : sah::binTail(C(id), cm, cinv, (float)nb, nb);
                    ++cnt[b];
                    bmn[b] = sah::vmin(bmn[b], amin[id]);
                    bmx[b] = sah::vmax(bmx[b], amax[id]);
                }
                split = sah::sweep(cnt.data(), bmn.data(), bmx.data(), rmn.data(), rmx.data(), nb, num, cost, areaInv, cm, ext);
            }
            std::vector<uint8_t> fl(num);
            for (uint32_t j = 0; j < num; ++j) { fl[j] = C(refs[start + j]) < split; nL += fl[j]; }
            median = nL == 0 || nL == num;
            if (!median) {   // closed-form two-pointer partition
                std::vector<uint32_t> slot(num);
                uint32_t Lb = 0;
                for (uint32_t j = 0; j < num; ++j) {
                    if (fl[j] && j >= nL) slot[nL - Lb - 1] = j;
                    Lb += fl[j];
                }
                Lb = 0;
                for (uint32_t j = 0; j < nL; ++j) {
                    if (!fl[j]) std::swap(refs[start + j], refs[start + slot[j - Lb]]);
                    else ++Lb;
                }
            }
        }
        const uint32_t nl = median ? num / 2 : nL, nr = num - nl;
        V4 b[8];
        for (int k = 0; k < 8; ++k) b[k] = (k & 1) ? V4{-INFINITY, -INFINITY, -INFINITY, -INFINITY} : V4{INFINITY, INFINITY, INFINITY, INFINITY};
        for (uint32_t j = 0; j < num; ++j) {
            const uint32_t id = refs[start + j];
            V4* B = j < nl ? b : b + 4;
            B[0] = sah::vmin(B[0], amin[id]); B[1] = sah::vmax(B[1], amax[id]);
            B[2] = sah::vmin(B[2], cen[id]); B[3] = sah::vmax(B[3], cen[id]);
        }
        const uint32_t li = index + 1, ri = index + nl * 2;
        float b0[6], b1[6];
        auto cbox = [&](uint32_t cn, uint32_t ref, V4 mn, V4 mx, float* bx) {
            if (cn == 1) sah::leafBox(&tri[9 * (size_t)ref], bx);
            else { bx[0] = mn.x; bx[1] = mn.y; bx[2] = mn.z; bx[3] = mx.x; bx[4] = mx.y; bx[5] = mx.z; }
        };
        cbox(nl, refs[start], b[0], b[1], b0);
        cbox(nr, refs[start + nl], b[4], b[5], b1);
        float* o = &nodes[16 * (size_t)index];
        o[0] = b0[0]; o[1] = b0[3]; o[2] = b0[1]; o[3] = b0[4];
        o[4] = b1[0]; o[5] = b1[3]; o[6] = b1[1]; o[7] = b1[4];
        o[8] = b0[2]; o[9] = b0[5]; o[10] = b1[2]; o[11] = b1[5];
        const int32_t ch[4] = {(int32_t)li, (int32_t)ri, 0, 0};
        std::memcpy(&o[12], ch, 16);
        if (nl == 1) { leaf(li, refs[start], so, po); depth = std::max(depth, (int)level + 1); }
        else node(b[0], b[1], b[2], b[3], start, nl, li, level + 1, so, po);
        if (nr == 1) { leaf(ri, refs[start + nl], so, po); depth = std::max(depth, (int)level + 1); }
        else node(b[4], b[5], b[6], b[7], start + nl, nr, ri, level + 1, so, po);
    }
};

static bool same(float a, float b) { return a == b ? true : std::memcmp(&a, &b, 4) == 0; }   // +0 == -0

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 20000;
    const unsigned seed = argc > 2 ? (unsigned)std::atoi(argv[2]) : 1;
    const int kind = argc > 3 ? std::atoi(argv[3]) : 0;
    std::mt19937 g(seed);
    std::uniform_real_distribution<float> U(-10.0f, 10.0f), S(-0.05f, 0.05f);
    std::vector<float> tri(9 * n);
    for (size_t k = 0; k < n; ++k) {
        float c[3];
        if (kind == 1) {   // grid: many equal centroid coordinates
            c[0] = (float)(k % 97); c[1] = (float)((k / 97) % 13) * 0.5f; c[2] = 0.0f;
        } else if (kind == 2) {   // a few clusters of identical triangles + a spread
            const int cl = (int)(k % 7);
            if (cl < 3) { c[0] = (float)cl; c[1] = 1.0f; c[2] = 2.0f; }
            else { c[0] = U(g); c[1] = U(g); c[2] = U(g); }
        } else {
            c[0] = U(g); c[1] = U(g) * 0.3f; c[2] = U(g) * 3.0f;
        }
        for (int v = 0; v < 3; ++v)
            for (int a = 0; a < 3; ++a) tri[9 * k + 3 * v + a] = c[a] + ((kind == 2 && (k % 7) < 3) ? 0.01f * (float)(v == a) : S(g));
    }
    std::vector<int32_t> so(n), po(n);
    for (size_t k = 0; k < n; ++k) { so[k] = (int32_t)(k % 3); po[k] = (int32_t)k; }
    BvhOut ref;
    if (!build_bvh(tri.data(), so.data(), po.data(), n, 10.0f, 64, true, 4, ref)) { std::puts("host build failed"); return 2; }
    const HostRcp& R = host_rcp_table();
    if (!R.ok) { std::puts("host rcp/dp rule check failed"); return 3; }
    Emu e{tri.data(), n, {}, {}, {}, {}, {}, &R, 64, 10.0f, true};
    e.amin.resize(n); e.amax.resize(n); e.cen.resize(n); e.refs.resize(n); e.nodes.assign(16 * (2 * n - 1), 0.0f);
    V4 smin{INFINITY, INFINITY, INFINITY, INFINITY}, smax{-INFINITY, -INFINITY, -INFINITY, -INFINITY}, cmin = smin, cmax = smax;
    for (size_t k = 0; k < n; ++k) {
        const float* p = &tri[9 * k];
        float mn[3], mx[3];
        for (int c = 0; c < 3; ++c) {
            const float a = p[c], bb = p[3 + c], cc = p[6 + c];
            const float m0 = (bb < a) ? bb : a, x0 = (a < bb) ? bb : a;
            mn[c] = (cc < m0) ? cc : m0;
            mx[c] = (x0 < cc) ? cc : x0;
        }
        e.amin[k] = V4{mn[0], mn[1], mn[2], 0.0f};
        e.amax[k] = V4{mx[0], mx[1], mx[2], 0.0f};
        e.cen[k] = V4{(mn[0] + mx[0]) * 0.5f, (mn[1] + mx[1]) * 0.5f, (mn[2] + mx[2]) * 0.5f, 0.0f};
        e.refs[k] = (uint32_t)k;
        smin = sah::vmin(smin, e.amin[k]); smax = sah::vmax(smax, e.amax[k]);
        cmin = sah::vmin(cmin, e.cen[k]); cmax = sah::vmax(cmax, e.cen[k]);
    }
    if (n == 1) e.leaf(0, 0, so.data(), po.data());
    else e.node(smin, smax, cmin, cmax, 0, (uint32_t)n, 0, 0, so.data(), po.data());
    size_t bad = 0, first = (size_t)-1;
    for (size_t i = 0; i < 16 * (2 * n - 1); ++i)
        if (!same(e.nodes[i], ref.nodes[i])) { if (!bad) first = i / 16; ++bad; }
    std::printf("n=%zu kind=%d rcp_bits=%d depth host=%d emu=%d mismatched floats=%zu first node=%lld\n", n, kind,
                R.bits, ref.depth, e.depth, bad, (long long)first);
    free_bvh(ref);
    return bad == 0 && e.depth == ref.depth ? 0 : 1;
}
