/*
 * ref_ssao.cpp -- TEST INFRASTRUCTURE ONLY (builds into oracle/_ref/).
 *
 * Renderer::post_process_ssao_SIMD (tp2/projets/renderer/renderer.cpp:1229-1434)
 * restated on the reference's own compiled SIMD helpers: __m256Point /
 * __m256Vector / _mm256_normalize / _mm256_dot_product / __m256Point::transform
 * (tp2/projets/SIMD/m256*.cpp), _mm256_reduction_ps (m256Utils.cpp), the 8-lane
 * and scalar xorshift generators (tp2/projets/renderer/xorshift.h) and the
 * scalar Vector / Point / Transform operators (tp2/src/vec.cpp, mat.cpp).
 * renderer.cpp itself includes <QImage> and cannot be compiled here, so the
 * loop structure is written out below: 8-pixel groups (skipped when every
 * lane is background), the scalar tail for render_width % 8 columns, the 7x7
 * blur and the QColor write-back.
 *
 * The one deliberate difference is the random stream: the reference seeds one
 * generator per OpenMP thread with std::rand(), which is not reproducible.
 * Here the 8 lanes of a group start from h_ssao_state(pixel of the lane) and the
 * scalar tail from h_ssao_state(pixel) -- the per-pixel streams that oracle.c
 * and the HIP kernel use.  QColor(int, int, int) + QImage::setPixelColor
 * (Qt 6: an out-of-range channel gives an invalid colour, which setPixelColor
 * ignores) are restated on ARGB32 words.
 *
 * Compiled with -mavx2 -mfma -ffp-contract=off: the reference's own
 * _mm256_fmadd_ps stays fused, nothing else is contracted.
 */
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include <immintrin.h>
#include <omp.h>

#include "m256Point.h"
#include "m256Utils.h"
#include "m256Vector.h"
#include "mat.h"
#include "vec.h"
#include "xorshift.h"

#include "orc_scene.h"

namespace {

uint32_t s_mix32(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU;
    x ^= x >> 15; x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// per-pixel stream (shared with oracle.c ssao_state and the HIP kernel)
uint32_t h_ssao_state(uint32_t pixel, uint32_t seed)
{
    uint32_t x = s_mix32(pixel * 0x9E3779B9u ^ seed ^ 0x5A0C1D3Bu);
    return x ? x : 0x9E3779B9u;
}

void to_xf(const float m[16], Transform& t)
{
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            t.m[i][j] = m[4 * i + j];
}

// x86 cvttss2si: NaN / out of range -> INT_MIN (the QColor arguments)
int f2i_x86(float f) { return _mm_cvtt_ss2si(_mm_set_ss(f)); }
// x86 cvttsd2si: the (int) of renderer.cpp:1392-1393's double products
int d2i_x86(double d) { return _mm_cvttsd_si32(_mm_set_sd(d)); }

}  // namespace

extern "C" int ref_ssao(const orc_scene* sc, const orc_settings* st, const float* zb, const float* nb, uint32_t* argb,
                        int32_t* ao_out)
{
    const int render_width = st->enable_ssaa ? st->image_width * st->ssaa_factor : st->image_width;
    const int render_height = st->enable_ssaa ? st->image_height * st->ssaa_factor : st->image_height;
    Transform proj;
    to_xf(sc->proj, proj);
    const float cam_fov = sc->cam_fov, cam_aspect = sc->cam_aspect;
    const float ssao_radius = st->ssao_radius;
    const int ssao_sample_count = st->ssao_sample_count;
    std::vector<int> ao_buffer((size_t)render_width * render_height, 0);

    const __m256 render_height_vec = _mm256_set1_ps((float)render_height);
    const __m256 render_width_vec = _mm256_set1_ps((float)render_width);
    const __m256 ones = _mm256_set1_ps(1);
    const __m256 twos = _mm256_set1_ps(2);
    const __m256 fov_multiplier = _mm256_set1_ps((float)std::tan(cam_fov / 2 / 180 * M_PI));

#pragma omp parallel for schedule(static)
    for (int y = 0; y < render_height; y++) {
        __m256 y_ndc = _mm256_sub_ps(_mm256_mul_ps(_mm256_div_ps(_mm256_set1_ps((float)y), render_height_vec), twos), ones);
        for (int x = 0; x + 8 <= render_width; x += 8) {
            const float* zrow = zb + (size_t)y * render_width;
            __m256 view_z = _mm256_loadu_ps(zrow + x);
            __m256 not_background = _mm256_cmp_ps(view_z, _mm256_set1_ps(INFINITY), _CMP_NEQ_OQ);
            if (_mm256_reduction_ps(not_background) == 0.0)
                continue;   // every lane background: no work, no random draws
            __m256 xs = _mm256_add_ps(_mm256_set_ps(7, 6, 5, 4, 3, 2, 1, 0), _mm256_set1_ps((float)x));
            __m256 x_ndc = _mm256_sub_ps(_mm256_mul_ps(_mm256_div_ps(xs, render_width_vec), twos), ones);
            __m256 view_ray_x = _mm256_mul_ps(x_ndc, _mm256_mul_ps(fov_multiplier, _mm256_set1_ps(cam_aspect)));
            __m256 view_ray_y = _mm256_mul_ps(y_ndc, fov_multiplier);
            __m256Point csp(_mm256_mul_ps(view_z, view_ray_x), _mm256_mul_ps(view_z, view_ray_y),
                            _mm256_mul_ps(view_z, _mm256_set1_ps(-1)));
            Vector nv[8];
            for (int j = 0; j < 8; j++) {
                const float* q = nb + 3 * ((size_t)y * render_width + x + j);
                nv[j] = Vector(q[0], q[1], q[2]);
            }
            __m256Vector normal = _mm256_normalize(__m256Vector(nv));
            uint32_t s[8];
            for (int j = 0; j < 8; j++)
                s[j] = h_ssao_state((uint32_t)(y * render_width + x + j), st->rng_seed);
            __m256_XorShiftGenerator gen(_mm256_set_epi32((int)s[7], (int)s[6], (int)s[5], (int)s[4], (int)s[3],
                                                          (int)s[2], (int)s[1], (int)s[0]));
            __m256i occlusion = _mm256_setzero_si256();
            for (int i = 0; i < ssao_sample_count; i++) {
                __m256 rx = gen.get_rand_bilateral();
                __m256 ry = gen.get_rand_bilateral();
                __m256 rz = gen.get_rand_bilateral();
                __m256Point sample = __m256Point(_mm256_normalize(__m256Vector(rx, ry, rz)));
                sample = sample * _mm256_add_ps(gen.get_rand_lateral(), _mm256_set1_ps(0.0001f));
                sample = sample * _mm256_set1_ps(ssao_radius);
                sample = sample + csp;
                __m256 facing = _mm256_dot_product(sample - csp, normal);
                __m256 flip = _mm256_and_ps(_mm256_cmp_ps(facing, _mm256_setzero_ps(), _CMP_LT_OQ), ones);
                __m256Vector back = 2 * (csp - sample);
                sample = sample + back * flip;
                __m256Point ndc = sample.transform(proj);
                __m256 half = _mm256_set1_ps(0.5);
                __m256i px = _mm256_cvtps_epi32(_mm256_mul_ps(_mm256_mul_ps(_mm256_add_ps(ndc._x, ones), half), render_width_vec));
                __m256i py = _mm256_cvtps_epi32(_mm256_mul_ps(_mm256_mul_ps(_mm256_add_ps(ndc._y, ones), half), render_height_vec));
                px = _mm256_max_epi32(_mm256_min_epi32(px, _mm256_cvtps_epi32(_mm256_sub_ps(render_width_vec, ones))),
                                      _mm256_set1_epi32(0));
                py = _mm256_max_epi32(_mm256_min_epi32(py, _mm256_cvtps_epi32(_mm256_sub_ps(render_height_vec, ones))),
                                      _mm256_set1_epi32(0));
                __m256i offs = _mm256_add_epi32(px, _mm256_mullo_epi32(py, _mm256_cvtps_epi32(render_width_vec)));
                __m256 geometry_depth = _mm256_mul_ps(_mm256_set1_ps(-1.0f), _mm256_i32gather_ps(zb, offs, sizeof(float)));
                __m256 occluded = ones;
                __m256 dz = _mm256_andnot_ps(_mm256_set1_ps(-0.0f), _mm256_sub_ps(geometry_depth, csp._z));
                occluded = _mm256_and_ps(occluded, _mm256_cmp_ps(dz, _mm256_set1_ps(ssao_radius), _CMP_LE_OQ));
                occluded = _mm256_and_ps(occluded, _mm256_cmp_ps(sample._z, geometry_depth, _CMP_LT_OQ));
                occluded = _mm256_and_ps(occluded, not_background);
                occlusion = _mm256_add_epi32(occlusion, _mm256_cvtps_epi32(occluded));
            }
            _mm256_storeu_si256((__m256i*)&ao_buffer[(size_t)y * render_width + x], occlusion);
        }

        // scalar tail (renderer.cpp:1363-1413)
        const float tan_half_fov = std::tan(radians(cam_fov / 2));
        for (int x = render_width - render_width % 8; x < render_width; x++) {
            float view_z = zb[(size_t)y * render_width + x];
            if (view_z == INFINITY)
                continue;
            float x_ndc = (float)x / render_width * 2 - 1;
            float y_ndc_s = (float)y / render_height * 2 - 1;
            float vrx = x_ndc * cam_aspect * tan_half_fov;
            float vry = y_ndc_s * tan_half_fov;
            Point csp(vrx * view_z, vry * view_z, -view_z);
            const float* q = nb + 3 * ((size_t)y * render_width + x);
            Vector normal = normalize(Vector(q[0], q[1], q[2]));
            XorShiftGenerator gen(h_ssao_state((uint32_t)(y * render_width + x), st->rng_seed));
            short int occ = 0;
            for (int i = 0; i < ssao_sample_count; i++) {
                float rx = gen.get_rand_bilateral();
                float ry = gen.get_rand_bilateral();
                float rz = gen.get_rand_bilateral();
                Point sample = Point(normalize(Vector(rx, ry, rz)));
                sample = sample * (gen.get_rand_lateral() + 0.0001f);
                sample = sample * ssao_radius;
                sample = sample + csp;
                if (dot(sample - csp, normal) < 0)
                    sample = sample + 2 * (csp - sample);
                Point ndc = proj(sample);
                int px = d2i_x86((ndc.x + 1) * 0.5 * render_width);
                int py = d2i_x86((ndc.y + 1) * 0.5 * render_height);
                px = std::min(std::max(0, px), render_width - 1);
                py = std::min(std::max(0, py), render_height - 1);
                float geometry_depth = -zb[(size_t)py * render_width + px];
                if (std::abs(geometry_depth - csp.z) > ssao_radius)
                    continue;
                if (sample.z < geometry_depth)
                    occ++;
            }
            ao_buffer[(size_t)y * render_width + x] = occ;
        }
    }

    // 7x7 blur applied to the image (renderer.cpp:1416-1431)
    const int blur_size = 7, half_blur = blur_size / 2;
#pragma omp parallel for schedule(static)
    for (int y = half_blur; y < render_height - half_blur; y++)
        for (int x = half_blur; x < render_width - half_blur; x++) {
            size_t o = (size_t)y * render_width + x;
            if (zb[o] == INFINITY)
                continue;
            int sum = 0;
            for (int oy = -half_blur; oy <= half_blur; oy++)
                for (int ox = -half_blur; ox <= half_blur; ox++)
                    sum += ao_buffer[(size_t)(y + oy) * render_width + x + ox];
            float mult = 1 - ((float)sum / (float)(blur_size * blur_size) / (float)ssao_sample_count * st->ssao_amount);
            uint32_t p = argb[o];
            int r = f2i_x86((int)((p >> 16) & 0xff) * mult);
            int g = f2i_x86((int)((p >> 8) & 0xff) * mult);
            int b = f2i_x86((int)(p & 0xff) * mult);
            if (r < 0 || r > 255 || g < 0 || g > 255 || b < 0 || b > 255)
                continue;   // invalid QColor: QImage::setPixelColor leaves the pixel
            argb[o] = 0xff000000u | ((uint32_t)r << 16) | ((uint32_t)g << 8) | (uint32_t)b;
        }
    if (ao_out)
        std::memcpy(ao_out, ao_buffer.data(), ao_buffer.size() * sizeof(int));
    return 0;
}
