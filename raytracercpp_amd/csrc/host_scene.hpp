// host_scene.hpp -- host-side scene setup (see host_scene.cpp).
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "rt_math.hpp"

namespace rt {
namespace mat {
void identity(float m[16]);
void translation(float x, float y, float z, float m[16]);
void scale(float x, float y, float z, float m[16]);
void rotation_x(float deg, float m[16]);
void rotation_y(float deg, float m[16]);
void rotation_z(float deg, float m[16]);
void compose(const float a[16], const float b[16], float out[16]);
void perspective(float fov, float aspect, float znear, float zfar, float m[16]);
bool inverse(const float in[16], float out[16]);
void transform_points(const float m[16], const float* pts, int64_t n, float* out);
}  // namespace mat

// Material as read from an .mtl (Material(Black()) defaults, materials.h:182-184)
struct ObjMaterial {
    float ambient[3] = {1.0f, 1.0f, 1.0f};
    float diffuse[3] = {0.0f, 0.0f, 0.0f};
    float specular[3] = {0.0f, 0.0f, 0.0f};
    float emission[3] = {0.0f, 0.0f, 0.0f};
    float reflection = 0.0f, roughness = 0.0f, ns = 0.0f, ni = 0.0f;
};

struct ObjData {
    std::vector<float> tri;     // [n][9]
    std::vector<int32_t> mat;   // [n]
    std::vector<float> uv;      // [n][6] when has_uv
    bool has_uv = false;
    std::vector<ObjMaterial> materials;
};

bool load_obj(const char* filename, const float xform[16], int mat_offset, ObjData& out, std::string& err);

}  // namespace rt
