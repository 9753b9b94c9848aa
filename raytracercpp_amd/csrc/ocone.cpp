// ocone.cpp -- the origin-cone grid (ocone.hpp): per cell, the cone of the stored normals of the
// triangles at risk for the cell's origins, found by a branch-and-bound walk of the wide BVH.
#include "ocone.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <queue>
#include <thread>

namespace rt {

namespace {

constexpr double PI = 3.14159265358979323846;

struct Cone {
    double a[3] = {0, 0, 0};   // unit axis
    double th = -1.0;          // half-angle (radians); < 0: empty, >= pi: every direction
};

double angle_between(const double* u, const double* v)
{
    // atan2 of |u x v| and u . v: accurate at every angle (unit vectors)
    const double cx = u[1] * v[2] - u[2] * v[1], cy = u[2] * v[0] - u[0] * v[2], cz = u[0] * v[1] - u[1] * v[0];
    return std::atan2(std::sqrt(cx * cx + cy * cy + cz * cz), u[0] * v[0] + u[1] * v[1] + u[2] * v[2]);
}

// the smallest cone holding both (enclosing-cone merge), widened by a relative 1e-12
Cone merge(const Cone& p, const Cone& q)
{
    if (p.th < 0)
        return q;
    if (q.th < 0)
        return p;
    if (p.th >= PI || q.th >= PI) {
        Cone c = p;
        c.th = PI;
        return c;
    }
    const double phi = angle_between(p.a, q.a);
    if (phi + q.th <= p.th)
        return p;
    if (phi + p.th <= q.th)
        return q;
    Cone c;
    c.th = 0.5 * (phi + p.th + q.th) * (1 + 1e-12) + 1e-15;
    if (c.th >= PI || !(phi > 1e-12)) {   // (phi ~ 0 with neither inside the other cannot happen but for rounding)
        c = p.th >= q.th ? p : q;
        c.th = std::min(PI, std::max(p.th, q.th) + phi + 1e-12);
        return c;
    }
    // rotate p.a towards q.a by (c.th - p.th): a = cos(x) p.a + sin(x) e, e the unit of q.a's part normal to p.a
    const double x = c.th - p.th;
    const double dp = p.a[0] * q.a[0] + p.a[1] * q.a[1] + p.a[2] * q.a[2];
    double e[3] = {q.a[0] - dp * p.a[0], q.a[1] - dp * p.a[1], q.a[2] - dp * p.a[2]};
    const double el = std::sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
    for (int i = 0; i < 3; i++)
        c.a[i] = std::cos(x) * p.a[i] + std::sin(x) * e[i] / el;
    const double al = std::sqrt(c.a[0] * c.a[0] + c.a[1] * c.a[1] + c.a[2] * c.a[2]);
    for (int i = 0; i < 3; i++)
        c.a[i] /= al;
    // the rotated axis' rounding: check both ends
    c.th = std::max(c.th, std::max(angle_between(c.a, p.a) + p.th, angle_between(c.a, q.a) + q.th) * (1 + 1e-12));
    return c;
}

// one child entry of the wide BVH (node v, slot j): what its triangles' planes and normals span
struct Agg {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    Cone plane;    // exact normals N = ab x ac of the non-degenerate triangles (the lemma's planes)
    Cone stored;   // stored normals n~ (Moller-Trumbore's Mdet), the non-zero ones, and the exact ones
    double lmax = 0, smin = INFINITY, s2min = INFINITY;   // the lemma's L, s, s2 (0: degenerate below)
    bool any = false;   // a triangle with a non-zero stored normal (one that can report at all)
};

void add_tri(Agg& g, const GTri& t)
{
    const double a[3] = {t.a[0], t.a[1], t.a[2]};
    for (int i = 0; i < 3; i++) {
        const double v0 = a[i], v1 = a[i] + (double)t.ab[i], v2 = a[i] + (double)t.ac[i];
        g.lo[i] = std::min(g.lo[i], std::min(v0, std::min(v1, v2)));
        g.hi[i] = std::max(g.hi[i], std::max(v0, std::max(v1, v2)));
    }
    const double nn = std::sqrt((double)t.n[0] * t.n[0] + (double)t.n[1] * t.n[1] + (double)t.n[2] * t.n[2]);
    if (nn == 0)
        return;   // Mdet = 0: never a hit
    g.any = true;
    Cone cs;
    if (!(nn < INFINITY)) {
        cs.th = PI;   // NaN / inf normal: no bound
    } else {
        for (int i = 0; i < 3; i++)
            cs.a[i] = t.n[i] / nn;
        cs.th = 1e-15;
    }
    g.stored = merge(g.stored, cs);
    const double x0 = t.ab[0], x1 = t.ab[1], x2 = t.ab[2], y0 = t.ac[0], y1 = t.ac[1], y2 = t.ac[2];
    const double c0 = x1 * y2 - x2 * y1, c1 = x2 * y0 - x0 * y2, c2 = x0 * y1 - x1 * y0;
    const double la = std::sqrt(x0 * x0 + x1 * x1 + x2 * x2), lc = std::sqrt(y0 * y0 + y1 * y1 + y2 * y2);
    const double cl = std::sqrt(c0 * c0 + c1 * c1 + c2 * c2);
    g.lmax = std::max(g.lmax, std::max(la, lc) * (1 + 1e-12));
    if (!(la * lc > 0x1p-100) || !(cl > 0x1p-50 * la * lc) || !(cl < INFINITY)) {
        g.smin = g.s2min = 0;   // degenerate: no H0 bound (always at risk, wbvh_risk_key)
        return;
    }
    const double ca = std::fabs(x0 * y0 + x1 * y1 + x2 * y2) / (la * lc);
    const double s2 = std::sqrt(std::fmax(0.0, (1.0 - std::fmin(1.0, ca + 1e-12)) / 2.0)) * (1 - 1e-9);
    g.smin = std::min(g.smin, cl / (la * lc) * (1 - 1e-9));
    g.s2min = std::min(g.s2min, s2);
    Cone cp;
    cp.a[0] = c0 / cl;
    cp.a[1] = c1 / cl;
    cp.a[2] = c2 / cl;
    cp.th = 1e-15;
    g.plane = merge(g.plane, cp);
    g.stored = merge(g.stored, cp);   // (the cell cones bound both normals: ocone_cell's front route reads N)
}

void add_agg(Agg& g, const Agg& c)
{
    for (int i = 0; i < 3; i++) {
        g.lo[i] = std::min(g.lo[i], c.lo[i]);
        g.hi[i] = std::max(g.hi[i], c.hi[i]);
    }
    g.plane = merge(g.plane, c.plane);
    g.stored = merge(g.stored, c.stored);
    g.lmax = std::max(g.lmax, c.lmax);
    g.smin = std::min(g.smin, c.smin);
    g.s2min = std::min(g.s2min, c.s2min);
    g.any |= c.any;
}

// the entries (ocone.hpp OConeEnt) bottom-up over the tree, cones rounded outwards
std::vector<OConeEnt> oc_entries(const WBvh& w)
{
    std::vector<Agg> agg(w.nodes.size() * W_WIDTH);
    std::vector<std::pair<uint32_t, bool>> st{{0u, false}};
    while (!st.empty()) {
        auto [v, done] = st.back();
        st.pop_back();
        const WNode& nd = w.nodes[v];
        if (!done) {
            st.push_back({v, true});
            for (int j = 0; j < W_WIDTH; j++)
                if (nd.child[j] != W_EMPTY && !(nd.child[j] & W_LEAF))
                    st.push_back({nd.child[j], false});
            continue;
        }
        for (int j = 0; j < W_WIDTH; j++) {
            const uint32_t ch = nd.child[j];
            Agg g;
            if (ch == W_EMPTY) {
            } else if (ch & W_LEAF) {
                const uint32_t first = (ch & ~W_LEAF) >> 3, cnt = (ch & 7u) + 1;
                for (uint32_t k = first; k < first + cnt; k++)
                    add_tri(g, w.tris[k]);
            } else {
                for (int i = 0; i < W_WIDTH; i++)
                    add_agg(g, agg[(size_t)ch * W_WIDTH + i]);
            }
            agg[(size_t)v * W_WIDTH + j] = g;
        }
    }
    std::vector<OConeEnt> E(agg.size());
    for (size_t e = 0; e < agg.size(); e++) {
        const Agg& g = agg[e];
        OConeEnt& o = E[e];
        for (int i = 0; i < 3; i++) {
            o.lo[i] = g.lo[i];
            o.hi[i] = g.hi[i];
            o.pa[i] = g.plane.a[i];
            o.sa[i] = g.stored.a[i];
        }
        // cos / sin of the half-angle, rounded outwards; a cone of pi / 2 or more has no bound (<= 0)
        auto cs = [](const Cone& c, double& co, double& si) {
            if (c.th < 0) {   // empty: a point cone (no triangle contributes)
                co = 1.0;
                si = 0.0;
            } else if (c.th >= 0.5 * PI * (1 - 1e-9)) {
                co = -1.0;
                si = 1.0;
            } else {
                co = std::cos(c.th) * (1 - 1e-12) - 1e-15;
                si = std::min(1.0, std::sin(c.th) * (1 + 1e-12) + 1e-15);
            }
        };
        cs(g.plane, o.pc, o.ps);
        cs(g.stored, o.sc, o.ss);
        if (g.stored.th >= PI)
            o.sc = -1.0;
        o.lmax = g.lmax;
        o.smin = g.smin;
        o.s2min = g.s2min;
        o.link = w.nodes[e / W_WIDTH].child[e % W_WIDTH];
        o.any = g.any ? 1u : 0u;
    }
    return E;
}

}  // namespace

void origin_cones_plan(const WBvh& w, float S, double QS, double reach, int max_dim, double beta_cap, OConeGrid& g,
                       OConeJob& job)
{
    g = OConeGrid();
    job = OConeJob();
    if (w.nodes.empty() || w.tris.empty() || max_dim < 1)
        return;
    job.ent = oc_entries(w);
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int j = 0; j < W_WIDTH; j++)
        if (job.ent[j].any)
            for (int i = 0; i < 3; i++) {
                lo[i] = std::min(lo[i], job.ent[j].lo[i]);
                hi[i] = std::max(hi[i], job.ent[j].hi[i]);
            }
    double ext = 0;
    for (int i = 0; i < 3; i++) {
        lo[i] -= reach;
        hi[i] += reach;
        ext = std::max(ext, hi[i] - lo[i]);
    }
    if (!(ext > 0) || !(ext < 1e30))
        return;
    // ih a float; cells of 1 / ih along every axis
    const float ihf = (float)(max_dim / ext);
    if (!(ihf > 0) || !(ihf < INFINITY))
        return;
    const double ih = ihf, h = 1.0 / ih;
    int64_t ncell = 1;
    for (int i = 0; i < 3; i++) {
        g.lo[i] = (float)lo[i];
        g.dim[i] = std::max(1, std::min(max_dim + 2, (int)std::ceil((hi[i] - (double)g.lo[i]) * ih) + 1));
        ncell *= g.dim[i];
    }
    g.ih = ihf;
    double om = 0;   // the largest |coordinate| of an origin in the grid
    for (int i = 0; i < 3; i++)
        om = std::max(om, std::max(std::fabs((double)g.lo[i]), std::fabs((double)g.lo[i] + g.dim[i] * h)));
    // the cell's ball: its half-diagonal, plus the float index computation's reach (o - lo and the
    // product each round once: 2^-24 relative of |o| + |lo|, and of the product <= dim)
    const double rnd = 0x1p-22 * (2 * om + (double)std::max(g.dim[0], std::max(g.dim[1], g.dim[2])) * h) + 1e-30;
    job.h = h;
    job.r = (0.5 * std::sqrt(3.0) * h + std::sqrt(3.0) * rnd) * (1 + 1e-9);
    job.slack = 1.01 * 0x1p-16 * (om + S);
    job.QS = QS;
    job.cos_cap = std::cos(beta_cap);
    // the cells within reach of a triangle (its box widened by reach)
    std::vector<uint8_t> mark((size_t)ncell, 0);
    for (size_t k = 0; k < w.tris.size(); k++) {
        const GTri& t = w.tris[k];
        int c0[3], c1[3];
        bool ok = true;
        for (int i = 0; i < 3; i++) {
            const double v0 = t.a[i], v1 = t.a[i] + (double)t.ab[i], v2 = t.a[i] + (double)t.ac[i];
            const double a = std::min(v0, std::min(v1, v2)) - reach, b = std::max(v0, std::max(v1, v2)) + reach;
            if (!(a <= b)) {
                ok = false;
                break;
            }
            c0[i] = std::max(0, (int)std::floor((a - g.lo[i]) * ih));
            c1[i] = std::min(g.dim[i] - 1, (int)std::floor((b - g.lo[i]) * ih));
        }
        if (!ok)
            continue;
        for (int z = c0[2]; z <= c1[2]; z++)
            for (int y = c0[1]; y <= c1[1]; y++)
                for (int x = c0[0]; x <= c1[0]; x++)
                    mark[((size_t)z * g.dim[1] + y) * g.dim[0] + x] = 1;
    }
    for (size_t i = 0; i < mark.size(); i++)
        if (mark[i])
            job.todo.push_back((uint32_t)i);
    g.computed = (int64_t)job.todo.size();
}

void build_origin_cones(const WBvh& w, float S, double QS, double reach, int max_dim, double beta_cap, int threads,
                        OConeGrid& g)
{
    auto t0 = std::chrono::steady_clock::now();
    OConeJob job;
    origin_cones_plan(w, S, QS, reach, max_dim, beta_cap, g, job);
    if (job.ent.empty())
        return;
    g.cells.assign((size_t)g.dim[0] * g.dim[1] * g.dim[2], uint2{0u, OC_NOSKIP << 16});
    if (threads <= 0)
        threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::atomic<size_t> next{0};
    auto work = [&]() {
        for (;;) {
            const size_t b = next.fetch_add(64);
            if (b >= job.todo.size())
                break;
            for (size_t i = b; i < std::min(job.todo.size(), b + 64); i++) {
                double c[3];
                ocone_center(g.lo, g.dim, job.h, job.todo[i], c);
                g.cells[job.todo[i]] = ocone_cell<OC_STACK>(job.ent.data(), w.tris.data(), c, job.r, job.slack, job.QS,
                                                             job.cos_cap);
            }
        }
    };
    std::vector<std::thread> pool;
    for (int i = 1; i < threads; i++)
        pool.emplace_back(work);
    work();
    for (auto& th : pool)
        th.join();
    origin_cones_count(g);
    g.ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void origin_cones_count(OConeGrid& g)
{
    g.empty = g.noskip = 0;
    for (const uint2& c : g.cells) {
        g.empty += (c.y >> 16) == OC_EMPTY;
        g.noskip += (c.y >> 16) == OC_NOSKIP;
    }
    g.noskip -= (int64_t)g.cells.size() - g.computed;   // (the cells out of reach)
}

}  // namespace rt
