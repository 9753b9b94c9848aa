// rt_math.hpp -- vector / colour / transform arithmetic shared by the host
// library and the gfx950 kernels.
//
// Every operator keeps the reference's operation order so that results are
// bit-identical to TomClabault/RayTracerCPP compiled with -ffp-contract=off:
//   Vector/Point ops ........ tp2/src/vec.cpp:41-177
//   Color ops ............... tp2/src/color.cpp:48-92
//   Point transform ......... tp2/src/mat.cpp:83-100
//   std::min / std::max ..... (b < a) ? b : a  /  (a < b) ? b : a
// The whole library is compiled with -ffp-contract=off and IEEE-exact
// (correctly rounded) fp32 division and square root.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define RT_HD __host__ __device__ __forceinline__

namespace rt {

struct v3 {
    float x, y, z;
};

// A load through the global address space: pointers read out of the KParams argument
// are generic, and a generic load is a FLAT instruction (counted in both vmcnt and
// lgkmcnt, so LDS waits also wait for it); this one is a global_load.
template <class T>
RT_HD T ldg(const T* p)
{
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(1))) T GT;
    return *(GT*)p;
#else
    return *p;
#endif
}

RT_HD v3 mk(float x, float y, float z) { return v3{x, y, z}; }
RT_HD v3 operator-(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_HD v3 operator+(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_HD v3 operator-(v3 a) { return mk(-a.x, -a.y, -a.z); }
// k * v and v * k both evaluate k*v.x, k*v.y, k*v.z (vec.cpp:102-110)
RT_HD v3 operator*(float k, v3 v) { return mk(k * v.x, k * v.y, k * v.z); }
RT_HD v3 operator*(v3 v, float k) { return mk(k * v.x, k * v.y, k * v.z); }
RT_HD float dot(v3 u, v3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
RT_HD v3 cross(v3 u, v3 v)
{
    return mk((u.y * v.z) - (u.z * v.y), (u.z * v.x) - (u.x * v.z), (u.x * v.y) - (u.y * v.x));
}
RT_HD float length2(v3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
RT_HD float length(v3 v) { return sqrtf(length2(v)); }
RT_HD v3 normalize(v3 v)
{
    float kk = 1 / length(v);
    return kk * v;
}

RT_HD float smin(float a, float b) { return (b < a) ? b : a; }
RT_HD float smax(float a, float b) { return (a < b) ? b : a; }
RT_HD float clamp01(float v) { return (v < 0.0f) ? 0.0f : ((1.0f < v) ? 1.0f : v); }

struct c3 {
    float r, g, b;
};
RT_HD c3 col(float r, float g, float b) { return c3{r, g, b}; }
RT_HD c3 operator+(c3 a, c3 b) { return col(a.r + b.r, a.g + b.g, a.b + b.b); }
RT_HD c3 operator*(c3 a, c3 b) { return col(a.r * b.r, a.g * b.g, a.b * b.b); }
RT_HD c3 operator*(c3 c, float k) { return col(c.r * k, c.g * k, c.b * k); }
RT_HD c3 operator/(c3 a, c3 b) { return col(a.r / b.r, a.g / b.g, a.b / b.b); }

// Transform::operator()(Point), mat.cpp:83-100 (m row-major, m[4*i+j] = m[i][j])
RT_HD v3 xform_point(const float* m, v3 p)
{
    float x = p.x, y = p.y, z = p.z;
    float xt = m[0] * x + m[1] * y + m[2] * z + m[3];
    float yt = m[4] * x + m[5] * y + m[6] * z + m[7];
    float zt = m[8] * x + m[9] * y + m[10] * z + m[11];
    float wt = m[12] * x + m[13] * y + m[14] * z + m[15];
    float w = 1.f / wt;
    if (wt == 1.f)
        return mk(xt, yt, zt);
    return mk(xt * w, yt * w, zt * w);
}

// x86-64 cvttss2si semantics (what the reference's float->int conversions
// compile to): NaN and out-of-range give INT_MIN.
RT_HD int f2i(float f)
{
    if (!(f > -2147483648.0f && f < 2147483648.0f))
        return (int)0x80000000;
    return (int)f;
}

// qRgb(r, g, b) (Qt), as used by ImageUtils::gkit_color_to_Qt_ARGB32_uint (imageUtils.h:149-152)
RT_HD uint32_t qrgb(int r, int g, int b)
{
    return 0xff000000u | ((uint32_t)(r & 0xff) << 16) | ((uint32_t)(g & 0xff) << 8) | (uint32_t)(b & 0xff);
}
RT_HD uint32_t color_to_argb(c3 c) { return qrgb(f2i(c.r * 255), f2i(c.g * 255), f2i(c.b * 255)); }

}  // namespace rt
