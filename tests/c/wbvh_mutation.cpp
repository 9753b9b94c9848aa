// The soundness metadata checkers must notice a wrong byte (wbvh.cpp check_wbvh / check_conditioning,
// check_risk_words).  Builds the octree and the wide BVH of a UV sphere with pole slivers plus a
// random sliver soup (librt_mi355x.so's own build), checks 0 violations, then, one at a time, moves a
// child's conditioning code to the unsafe side (smin / s2 up, sth / lmax / rho down) and a risk word's
// key up / its at-risk box in, and requires each change to be reported.  Prints "ok <mutations>".
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../../raytracercpp_amd/csrc/wbvh.hpp"

using namespace rt;

static void sphere(std::vector<float>& t, int nu, int nv, float r)
{
    auto P = [&](int i, int j, float* o) {
        const double th = M_PI * j / nv, ph = 2 * M_PI * (i % nu) / nu;
        o[0] = (float)(r * std::sin(th) * std::cos(ph));
        o[1] = (float)(r * std::cos(th));
        o[2] = (float)(r * std::sin(th) * std::sin(ph) - 3.0);
    };
    for (int i = 0; i < nu; i++)
        for (int j = 0; j < nv; j++) {
            float a[3], b[3], c[3], d[3];
            P(i, j, a), P(i + 1, j, b), P(i + 1, j + 1, c), P(i, j + 1, d);
            for (float* v : {a, b, c, a, c, d})
                t.insert(t.end(), v, v + 3);
        }
}

int main()
{
    std::vector<float> tri;
    sphere(tri, 160, 80, 1.2f);
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(-1.0f, 1.0f);
    for (int k = 0; k < 2000; k++) {   // slivers
        const float cx = 3 * U(rng), cy = 3 * U(rng), cz = -6 + U(rng), ex = U(rng), ey = U(rng), ez = U(rng);
        const float f = 0.5f + 0.5f * U(rng);
        const float v[9] = {cx, cy, cz, cx + 0.2f * ex, cy + 0.2f * ey, cz + 0.2f * ez,
                            cx + 0.2f * f * ex + 1e-4f * U(rng), cy + 0.2f * f * ey, cz + 0.2f * f * ez};
        tri.insert(tri.end(), v, v + 9);
    }
    const int64_t n = (int64_t)tri.size() / 9;
    FlatOctree f;
    build_flat_octree(tri.data(), n, 12, 40, f);
    WBvh w;
    build_wbvh(f, w);
    int64_t v0 = check_wbvh(f, w);
    if (v0 != 0) {
        std::printf("FAIL: %lld violations on the unmodified tree\n", (long long)v0);
        return 1;
    }
    int mutations = 0;
    // conditioning codes: byte b of ext (0 smin, 1 s2, 2 sth, 3 lmax) or ext2 byte 0 (rho); +1 for a lower
    // bound moved up, -1 for an upper bound moved down
    struct Field {
        int word, shift, dir;
        const char* name;
    } fields[5] = {{0, 0, +1, "smin"}, {0, 8, +1, "s2"}, {0, 16, -1, "sth"}, {0, 24, -1, "lmax"}, {1, 0, -1, "rho"}};
    for (const Field& F : fields) {
        int tried = 0, caught = 0;
        for (size_t v = 0; v < w.nodes.size() && tried < 6; v += 1 + w.nodes.size() / 97) {
            for (int j = 0; j < W_WIDTH && tried < 6; j++) {
                if (w.nodes[v].child[j] == W_EMPTY)
                    continue;
                uint32_t& word = F.word == 0 ? w.nodes[v].ext[j] : w.nodes[v].ext2[j];
                const uint32_t code = (word >> F.shift) & 0xffu;
                // a move of two codes (a quarter octave) to the unsafe side, within 1..254; lower bounds
                // from 2^-10 up (code 175), where the build's own margins (sin_at_a_lb's 2^-50, s2's
                // 1e-12 on the cosine) are far below a quarter octave, so the moved code exceeds the
                // true minimum
                if (F.dir > 0 ? (code < 175 || code > 252) : (code < 3 || code == 255))
                    continue;
                const uint32_t saved = word;
                word = (word & ~(0xffu << F.shift)) | ((code + 2 * F.dir) << F.shift);
                tried++;
                caught += check_wbvh(f, w) > 0;
                word = saved;
            }
        }
        if (tried == 0 || caught != tried) {
            std::printf("FAIL: %s: %d of %d corrupted codes reported\n", F.name, caught, tried);
            return 1;
        }
        mutations += tried;
    }
    // risk words of a camera grazing the sphere's silhouette
    const float lo[3] = {f.nodes[0].dn[0], f.nodes[0].dn[1], f.nodes[0].dn[2]};
    const float hi[3] = {f.nodes[0].df[0], f.nodes[0].df[1], f.nodes[0].df[2]};
    float S = 0;
    for (int a = 0; a < 3; a++)
        S = std::max(S, std::max(std::fabs(lo[a]), std::fabs(hi[a])));
    const float cam[3] = {1.2f, 0.0f, 0.5f}, light[3] = {3, 3, 2};
    const WRiskArgs A = wbvh_risk_args(lo, hi, S, cam, light, W_QS_CLOSEST, W_QS_SHADOW);
    std::vector<float> lbox(6 * w.tris.size());
    for (size_t k = 0; k < w.tris.size(); k++)
        for (int a = 0; a < 3; a++) {
            lbox[6 * k + a] = f.nodes[w.leaf_of_k[k]].dn[a];
            lbox[6 * k + 3 + a] = f.nodes[w.leaf_of_k[k]].df[a];
        }
    std::vector<uint64_t> risk;
    wbvh_risk_host(w, lbox, A, 0, risk);
    wbvh_risk_host(w, lbox, A, 1, risk);
    for (int sel = 0; sel < 2; sel++)
        if (check_risk_words(f, w, A, sel, risk.data()) != 0) {
            std::printf("FAIL: risk words %d violate on the unmodified tree\n", sel);
            return 1;
        }
    int tried = 0, caught = 0;
    for (size_t i = 0; i < risk.size() && tried < 40; i += 1 + risk.size() / 4001) {
        const int sel = (int)((i >> 2) & 1);
        const uint64_t word = risk[i];
        const float K = wrisk_key(word);
        if (!(K < INFINITY))
            continue;
        // (1) the key up by a factor 4 (or from 0 to a positive one)
        risk[i] = wrisk_pack(K > 0 ? 4 * K : 1e-3f, word);
        tried++;
        caught += check_risk_words(f, w, A, sel, risk.data()) > 0;
        // (2) the at-risk box's high x byte down (when the box spans more than a code and the entry has no
        // rho slack: the query widens the box by rho, so a byte moved within rho is still sound)
        const uint32_t hx = (uint32_t)((word >> 24) & 0xffu), lx = (uint32_t)(word & 0xffu);
        risk[i] = word;
        if (hx > lx + 2 && (w.nodes[i >> 3].ext2[i & 3] & 0xffu) == 0) {
            risk[i] = (word & ~(0xffull << 24)) | ((uint64_t)(hx - 2) << 24);
            tried++;
            caught += check_risk_words(f, w, A, sel, risk.data()) > 0;
        }
        risk[i] = word;
    }
    if (tried < 10 || caught != tried) {
        std::printf("FAIL: risk words: %d of %d corrupted words reported\n", caught, tried);
        return 1;
    }
    mutations += tried;
    std::printf("ok %d\n", mutations);
    return 0;
}
