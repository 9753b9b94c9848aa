// kdop_certifies (wbvh.hpp): the decision through an approximate reciprocal must be the
// correctly rounded one's (kdop_certifies_exact, BoundingVolume::intersect bvh.h:79-105) for every
// input.  Host build with a reciprocal hook that is off by up to +-4 ulps (the device's
// v_rcp_f32 is within 1), on random k-DOPs and rays, on comparisons within a few ulps of the
// decision (the fallback path), on tiny, zero and huge denominators.  Prints "ok <n>" or the
// first mismatch.
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>

static uint64_t g_state = 0x9E3779B97F4A7C15ull;
static int g_ulps = 4;
static float rcp_hook(float a)
{
    float r = 1.0f / a;
    g_state = g_state * 6364136223846793005ull + 1442695040888963407ull;
    int k = (int)((g_state >> 33) % (uint64_t)(2 * g_ulps + 1)) - g_ulps;
    for (; k > 0; k--) r = std::nextafter(r, INFINITY);
    for (; k < 0; k++) r = std::nextafter(r, -INFINITY);
    return r;
}
#define RT_TEST_RCP_HOOK rcp_hook
#include "../../raytracercpp_amd/csrc/wbvh.hpp"

int main()
{
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<float> U(-1.0f, 1.0f);
    long n = 0, fallback_band = 0;
    for (int it = 0; it < 2000000; it++) {
        rt::GNode g;
        std::memset(&g, 0, sizeof(g));
        const float scale = std::ldexp(1.0f, (int)(rng() % 41) - 20);
        const float cx = U(rng) * scale, cy = U(rng) * scale, cz = U(rng) * scale;
        for (int i = 0; i < rt::NPLANES; i++) {
            const float c = cx * rt::PLANE_N[i][0] + cy * rt::PLANE_N[i][1] + cz * rt::PLANE_N[i][2];
            const float a = std::fabs(U(rng)) * scale, b = std::fabs(U(rng)) * scale;
            g.dn[i] = c - a;
            g.df[i] = c + b;
        }
        rt::v3 o = rt::mk(U(rng) * 4 * scale, U(rng) * 4 * scale, U(rng) * 4 * scale);
        rt::v3 d = rt::mk(U(rng), U(rng), U(rng));
        const int kind = (int)(rng() % 8);
        if (kind == 1) d.x = 0.0f;                                   // a skipped plane
        if (kind == 2) d.y = std::ldexp(U(rng), -110);                // a denominator below 2^-100
        if (kind == 3) d = rt::mk(d.x * 1e-30f, d.y * 1e-30f, d.z);   // tiny components
        // t: random, or at the exact path's own t_near / t_far within a few ulps (close calls)
        float tn = -INFINITY, tf = INFINITY;
        for (int i = 0; i < rt::NPLANES; i++) {
            rt::v3 pn = rt::mk(rt::PLANE_N[i][0], rt::PLANE_N[i][1], rt::PLANE_N[i][2]);
            float den = rt::dot(pn, d), num = rt::dot(pn, o);
            if (den == 0.0f) continue;
            float d0 = (g.dn[i] - num) / den, d1 = (g.df[i] - num) / den;
            tn = std::fmax(tn, std::fmin(d0, d1));
            tf = std::fmin(tf, std::fmax(d0, d1));
        }
        float t = U(rng) * 8 * scale;
        if (kind >= 4 && std::isfinite(tn)) {
            t = tn;
            for (int k = (int)(rng() % 9) - 4; k != 0; k += k > 0 ? -1 : 1)
                t = std::nextafter(t, k > 0 ? INFINITY : -INFINITY);
            fallback_band++;
        }
        const bool fast = rt::kdop_certifies(g, o, d, t), exact = rt::kdop_certifies_exact(g, o, d, t);
        n++;
        if (fast != exact) {
            std::printf("mismatch at %d: fast %d exact %d t %a tn %a tf %a\n", it, fast, exact, t, tn, tf);
            return 1;
        }
    }
    std::printf("ok %ld (%ld near t_near)\n", n, fallback_band);
    return 0;
}
