// The rounding lemma behind the sound child test of the wide query (wbvh.hpp
// wbvh_closest, wq_h0), checked directly on Moller-Trumbore's own float arithmetic (mt_record, the
// expressions of triangle.cpp:25-91, on records built as octree.cpp make_gtri builds them).  For every
// hit mt_record accepts, with u = 2^-24, q = |cos(n, d)|, s = sin(alpha) (alpha: the angle at a),
// s2 = sin(alpha' / 2) (alpha' = min(alpha, pi - alpha)), L = max(|ab|, |ac|), all for the exact
// triangle (a, a + ab, a + ac) of the record in x87 long double, and D the query's bound on the
// origin's distance: in (a) from every point of the triangle (the query's Dn, the distance to the
// farthest corner of the node's frame, bounds it; here D = the farthest vertex), in (b) from a:
//   (a) when B = 7.21u / (q s) + 2.01u <= 1/2: the reported point p' = o + t' d lies within
//       R = (A + B D) / (1 - B), A = u (30.4 D + 14.4 L) / (q s) + u (4.02 L + 2.01 D), of the triangle,
//       and within eta = u (5 + 8 / s) (2 D + R) of its plane;
//   (b) for every q: the origin lies within H0 = 1.01 [q (2L + D) + u (24.2 L + 48 D) / s +
//       u (30 L + 12 D + 24 D / s) / s2] of the plane (wq_h0 with QS = q, the strongest form).
// Random triangles (slivers with sines down to 1e-7 and obtuse ones, scales 2^-6 .. 2^6, offsets up to
// 8x the scale), rays aimed at points in and around them with q log-uniform in [1e-10, 1] (so Q = q s
// covers 1e-9 .. 1 and below), origins at 0.1 .. 300 edge lengths.  The same hits are also checked
// against the float functions the kernels evaluate (wq_reach, wq_split, wq_eta, wq_h0 on float bounds of
// the exact quantities).  Prints "ok <acceptances> <max ratio dist/R> <max plane/eta> <max origin/H0> ...
// float-bounds <|p'-P'|/E> <lat/Rlat> <plane/eta> <origin/H0>" or the first violation.
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "../../raytracercpp_amd/csrc/wbvh.hpp"

typedef long double ld;
struct L3 {
    ld x, y, z;
};
static L3 l3(ld x, ld y, ld z) { return L3{x, y, z}; }
static L3 operator-(L3 a, L3 b) { return l3(a.x - b.x, a.y - b.y, a.z - b.z); }
static L3 operator+(L3 a, L3 b) { return l3(a.x + b.x, a.y + b.y, a.z + b.z); }
static L3 operator*(L3 a, ld k) { return l3(a.x * k, a.y * k, a.z * k); }
static ld dotl(L3 a, L3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static L3 crossl(L3 a, L3 b) { return l3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static ld lenl(L3 a) { return sqrtl(dotl(a, a)); }

// closest point of triangle (a, b, c) to p (Ericson, Real-Time Collision Detection 5.1.5)
static L3 closest_on_tri(L3 p, L3 a, L3 b, L3 c)
{
    const L3 ab = b - a, ac = c - a, ap = p - a;
    const ld d1 = dotl(ab, ap), d2 = dotl(ac, ap);
    if (d1 <= 0 && d2 <= 0) return a;
    const L3 bp = p - b;
    const ld d3 = dotl(ab, bp), d4 = dotl(ac, bp);
    if (d3 >= 0 && d4 <= d3) return b;
    const ld vc = d1 * d4 - d3 * d2;
    if (vc <= 0 && d1 >= 0 && d3 <= 0) return a + ab * (d1 / (d1 - d3));
    const L3 cp = p - c;
    const ld d5 = dotl(ab, cp), d6 = dotl(ac, cp);
    if (d6 >= 0 && d5 <= d6) return c;
    const ld vb = d5 * d2 - d1 * d6;
    if (vb <= 0 && d2 >= 0 && d6 <= 0) return a + ac * (d2 / (d2 - d6));
    const ld va = d3 * d6 - d5 * d4;
    if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) return b + (c - b) * ((d4 - d3) / ((d4 - d3) + (d5 - d6)));
    const ld den = 1 / (va + vb + vc);
    return a + ab * (vb * den) + ac * (vc * den);
}

int main(int argc, char** argv)
{
    const long target = argc > 1 ? std::atol(argv[1]) : 10000000L;
    const double far = argc > 2 ? std::atof(argv[2]) : 300.0;   // origins at 0.1 .. far edge lengths
    const unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::atomic<long> accepted{0}, samples{0};
    std::atomic<int> failed{0};
    std::mutex mu;
    ld worst[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    long bins[10] = {};   // acceptances by floor(-log10 Q), Q = q s
    auto work = [&](unsigned tid) {
        std::mt19937_64 rng(0x5EED0000ull + tid);
        std::uniform_real_distribution<double> U(0.0, 1.0);
        auto logu = [&](double lo, double hi) { return std::exp(std::log(lo) + U(rng) * (std::log(hi) - std::log(lo))); };
        auto unit = [&]() {
            std::normal_distribution<double> N(0.0, 1.0);
            double x = N(rng), y = N(rng), z = N(rng), l = std::sqrt(x * x + y * y + z * z);
            return l3(x / l, y / l, z / l);
        };
        ld w[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        long lb[10] = {};
        while (accepted.load(std::memory_order_relaxed) < target && !failed.load()) {
            samples++;
            const double S = std::ldexp(1.0, (int)(rng() % 13) - 6);
            // the triangle: edges at a of lengths la, lc and angle alpha (slivers, obtuse slivers)
            const double la = S * logu(0.01, 1.0), lc = S * logu(0.01, 1.0);
            double alpha = logu(1e-7, 1.5707963267948966);
            if (rng() % 4 == 0)
                alpha = 3.141592653589793 - alpha;
            const L3 e1 = unit();
            L3 e2 = unit();
            e2 = e2 - e1 * dotl(e1, e2);
            e2 = e2 * (1 / lenl(e2));
            const L3 a0 = l3((2 * U(rng) - 1) * 8 * S, (2 * U(rng) - 1) * 8 * S, (2 * U(rng) - 1) * 8 * S);
            const L3 b0 = a0 + e1 * la, c0 = a0 + (e1 * std::cos(alpha) + e2 * std::sin(alpha)) * lc;
            const rt::v3 va = rt::mk((float)a0.x, (float)a0.y, (float)a0.z), vb = rt::mk((float)b0.x, (float)b0.y, (float)b0.z),
                         vc = rt::mk((float)c0.x, (float)c0.y, (float)c0.z);
            // octree.cpp make_gtri
            rt::GTri T;
            const rt::v3 ab = vb - va, ac = vc - va, nn = rt::cross(vb - va, vc - va);
            T.a[0] = va.x; T.a[1] = va.y; T.a[2] = va.z;
            T.ab[0] = ab.x; T.ab[1] = ab.y; T.ab[2] = ab.z;
            T.ac[0] = ac.x; T.ac[1] = ac.y; T.ac[2] = ac.z;
            T.n[0] = nn.x; T.n[1] = nn.y; T.n[2] = nn.z;
            const L3 A = l3(va.x, va.y, va.z), AB = l3(ab.x, ab.y, ab.z), AC = l3(ac.x, ac.y, ac.z);
            const L3 NX = crossl(AB, AC);
            const ld nl = lenl(NX), lab = lenl(AB), lac = lenl(AC);
            if (!(nl > 0) || !(lab > 0) || !(lac > 0))
                continue;
            const L3 nh = NX * (1 / nl);
            // a target point in and around the triangle, a direction at |cos(n, d)| = q, facing it
            const double bu = -0.05 + 1.1 * U(rng), bv = -0.05 + 1.1 * U(rng);
            const L3 P = A + AB * bu + AC * bv;
            const double q = logu(1e-10, 1.0);
            L3 tdir = unit();
            tdir = tdir - nh * dotl(nh, tdir);
            const ld tl = lenl(tdir);
            if (!(tl > 0))
                continue;
            tdir = tdir * (1 / tl);
            const L3 d0 = tdir * std::sqrt(1 - q * q) + nh * (-q);
            const L3 o0 = P - d0 * (std::max(la, lc) * logu(0.1, far));
            const rt::v3 o = rt::mk((float)o0.x, (float)o0.y, (float)o0.z), d = rt::mk((float)d0.x, (float)d0.y, (float)d0.z);
            float t, u, v;
            if (!rt::mt_record(T, o, d, t, u, v) || !std::isfinite(t))
                continue;
            accepted++;
            // exact quantities of the accepted hit
            const L3 O = l3(o.x, o.y, o.z), Dd = l3(d.x, d.y, d.z);
            const ld qq = fabsl(dotl(Dd, nh)) / lenl(Dd);
            const ld s = nl / (lab * lac);
            const ld ca = fabsl(dotl(AB, AC)) / (lab * lac);
            const ld s2 = sqrtl(fmaxl(0.0L, (1 - ca) / 2));
            const ld D = lenl(O - A), L = fmaxl(lab, lac);
            const ld Dv = fmaxl(D, fmaxl(lenl(O - (A + AB)), lenl(O - (A + AC))));
            const ld uu = 0x1p-24L;
            const L3 Pp = O + Dd * (ld)t;
            const ld pl = fabsl(dotl(Pp - A, nh));
            const ld od = fabsl(dotl(O - A, nh));
            const ld Q = qq * s;
            const int bin = Q > 0 ? std::min(9, std::max(0, (int)std::floor(-std::log10((double)Q)))) : 9;
            lb[bin]++;
            const ld H0 = 1.01L * (qq * (2 * L + D) + uu * (24.2L * L + 48 * D) / s + uu * (30 * L + 12 * D + 24 * D / s) / s2);
            ld r2 = od / H0, r0 = 0, r1 = 0, r3 = 0, r4 = 0;
            bool bad = !(od <= H0);
            // case (a), wbvh.hpp wq_reach (the correlated bound): G >= q - 5.85u / s,
            // isG >= 1 / (s G), iG >= 1 / G
            const ld X = s * qq - 5.85L * uu;
            if (X > 0) {
                const ld isG = 1 / X, iG = s * isG;
                const ld beta = 8.85L * uu * isG + 2.011L * uu;
                if (beta <= 0.5L) {
                    const ld E = (8.85L * uu * (1 + uu) * L * isG + 10.87L * uu * Dv * iG + 43 * uu * uu * Dv * isG +
                                  2.011L * uu * (Dv + L)) * (1 + 2 * beta);
                    const ld kq = (1 + 2.83L * uu * isG) * (1 + 5.85L * uu * isG);
                    const ld eta = (2.83L * uu * ((1 + uu) * L + E) * isG + (3.01L * (Dv + E) + 4.02L * Dv) * uu * kq +
                                    2.011L * uu * (Dv + E)) / (1 - 3.02L * uu * iG - 9 * uu * uu * isG);
                    // P' = a + u' ab + v' ac (MT's accepted barycentrics), |p' - P'| <= E
                    const L3 Pq = A + AB * (ld)u + AC * (ld)v;
                    const ld pP = lenl(Pp - Pq);
                    const L3 cp = closest_on_tri(Pp, A, A + AB, A + AC);
                    const ld dist = lenl(Pp - cp);
                    r0 = dist / (E + 2.02L * uu * L);
                    r3 = pP / E;
                    r1 = pl / eta;
                    bad |= !(dist <= E + 2.02L * uu * L) || !(pP <= E) || !(pl <= eta);
                    // wq_split: p' - P' = lat + par with par along d, |par| <= Rpar, |lat| <= Rlat, i.e. P' lies
                    // within Rlat of the line's segment [p' - Rpar d^, p' + Rpar d^]
                    const ld kn = 1 + 2.83L * uu * isG;
                    const ld Rlat = 8.85L * uu * ((1 + uu) * L + E) * isG + 3.02L * uu * ((1 + uu) * L + E) * iG * kn +
                                    3.84L * uu * Dv * iG + 23.2L * uu * uu * Dv * isG + 2.012L * uu * L;
                    const ld Rpar = (4.02L * D + 3.01L * (Dv + E)) * uu * iG * kn + 2.011L * uu * (Dv + E);
                    const ld dl = lenl(Dd);
                    const L3 dh = Dd * (1 / dl);
                    const ld x = std::max(-Rpar, std::min(Rpar, dotl(Pq - Pp, dh)));
                    const ld lat = lenl(Pq - (Pp + dh * x));
                    r4 = lat / Rlat;
                    bad |= !(lat <= Rlat);
                }
            }
            // the SHIPPED float bounds (wbvh.hpp wq_reach / wq_split / wq_eta / wq_h0, as the query evaluates
            // them) on float bounds of the exact quantities (q, s, s2 rounded down; L, D rounded up): a typo
            // or a rounding slip in the constants the kernels run would show here, not only in an oracle frame
            {
                auto dn = [](ld x) { float f = (float)x; return (ld)f > x ? std::nextafterf(f, 0.0f) : f; };
                auto up = [](ld x) { float f = (float)x; return (ld)f < x ? std::nextafterf(f, INFINITY) : f; };
                const float qf = dn(qq), sf = dn(s), s2f = dn(s2), Lf = up(L), Df = up(D), Dvf = up(Dv);
                const rt::WReach wr = rt::wq_reach(qf, sf, Lf, Dvf);
                if (wr.E < INFINITY) {
                    const L3 Pq = A + AB * (ld)u + AC * (ld)v;
                    const L3 cp = closest_on_tri(Pp, A, A + AB, A + AC);
                    const ld dist = lenl(Pp - cp), pP = lenl(Pp - Pq);
                    float Rlat, Rpar;
                    rt::wq_split(wr, Lf, Dvf, Rlat, Rpar);
                    const float eta = rt::wq_eta(wr, Lf, Dvf);
                    const ld dl = lenl(Dd);
                    const L3 dh = Dd * (1 / dl);
                    const ld x = std::max(-(ld)Rpar, std::min((ld)Rpar, dotl(Pq - Pp, dh)));
                    const ld lat = lenl(Pq - (Pp + dh * x));
                    w[5] = fmaxl(w[5], pP / wr.E);
                    w[6] = fmaxl(w[6], lat / Rlat);
                    w[7] = fmaxl(w[7], pl / eta);
                    bad |= !(pP <= wr.E) || !(dist <= wr.E + 2.02L * uu * L) || !(lat <= Rlat) || !(pl <= eta);
                }
                // case (b) with QS = q rounded up (the strongest form the kernels can evaluate)
                const float h0 = rt::wq_h0(up(qq), Lf, Df, sf, s2f);
                w[8] = fmaxl(w[8], od / h0);
                bad |= !(od <= h0);
            }
            w[0] = fmaxl(w[0], r0);
            w[1] = fmaxl(w[1], r1);
            w[2] = fmaxl(w[2], r2);
            w[3] = fmaxl(w[3], r3);
            w[4] = fmaxl(w[4], r4);
            if (bad && !failed.exchange(1)) {
                std::lock_guard<std::mutex> g(mu);
                std::printf("VIOLATION q %.6Lg s %.6Lg s2 %.6Lg D %.6Lg L %.6Lg t %.9g u %.9g v %.9g: dist/R %.6Lg "
                            "plane/eta %.6Lg origin/H0 %.6Lg |p'-P'|/E %.6Lg lat/Rlat %.6Lg\n",
                            qq, s, s2, D, L, t, u, v, r0, r1, r2, r3, r4);
            }
        }
        std::lock_guard<std::mutex> g(mu);
        for (int i = 0; i < 9; i++)
            worst[i] = fmaxl(worst[i], w[i]);
        for (int i = 0; i < 10; i++)
            bins[i] += lb[i];
    };
    std::vector<std::thread> th;
    for (unsigned k = 0; k < nth; k++)
        th.emplace_back(work, k);
    for (auto& x : th)
        x.join();
    if (failed.load())
        return 1;
    std::printf("ok %ld %.4Lg %.4Lg %.4Lg %.4Lg %.4Lg samples %ld Q-decades", accepted.load(), worst[0], worst[1],
                worst[2], worst[3], worst[4], samples.load());
    for (int i = 0; i < 10; i++)
        std::printf(" %ld", bins[i]);
    std::printf(" float-bounds %.4Lg %.4Lg %.4Lg %.4Lg\n", worst[5], worst[6], worst[7], worst[8]);
    return 0;
}
