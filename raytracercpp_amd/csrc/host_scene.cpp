// host_scene.cpp -- host-side scene setup the hot path depends on:
//   * Transform algebra (tp2/src/mat.cpp restated: Perspective, Gauss-Jordan
//     inverse, rotations, composition, point transform);
//   * OBJ / MTL loading with the reference's exact fan triangulation and vertex
//     de-duplication order (read_meshio_data, tp2/src/mesh_io.cpp:426-591;
//     read_materials_mtl, :213-304) and MeshIOUtils::create_triangles
//     (tp2/projets/utils/meshIOUtils.cpp:4-30), so triangle indices (the
//     hit-ID parity key) match the reference.
// Compiled with -ffp-contract=off like the rest of the library.
#include "host_scene.hpp"

#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <map>
#include <string>

namespace rt {
namespace mat {

static float radians(float deg) { return ((float)M_PI / 180) * deg; }   // mat.cpp:13-16

void identity(float m[16])
{
    for (int i = 0; i < 16; i++) m[i] = (i % 5 == 0) ? 1.0f : 0.0f;
}

void translation(float x, float y, float z, float m[16])
{
    identity(m);
    m[3] = x;
    m[7] = y;
    m[11] = z;
}

void scale(float x, float y, float z, float m[16])
{
    identity(m);
    m[0] = x;
    m[5] = y;
    m[10] = z;
}

void rotation_x(float a, float m[16])   // mat.cpp:208-218
{
    float s = sinf(radians(a)), c = cosf(radians(a));
    identity(m);
    m[5] = c; m[6] = -s;
    m[9] = s; m[10] = c;
}

void rotation_y(float a, float m[16])   // mat.cpp:220-230
{
    float s = sinf(radians(a)), c = cosf(radians(a));
    identity(m);
    m[0] = c; m[2] = s;
    m[8] = -s; m[10] = c;
}

void rotation_z(float a, float m[16])   // mat.cpp:232-242
{
    float s = sinf(radians(a)), c = cosf(radians(a));
    identity(m);
    m[0] = c; m[1] = -s;
    m[4] = s; m[5] = c;
}

void compose(const float a[16], const float b[16], float out[16])   // mat.cpp:363-371
{
    float m[16];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            m[4 * i + j] = a[4 * i + 0] * b[0 + j] + a[4 * i + 1] * b[4 + j] + a[4 * i + 2] * b[8 + j] +
                           a[4 * i + 3] * b[12 + j];
    std::memcpy(out, m, sizeof(m));
}

void perspective(float fov, float aspect, float znear, float zfar, float m[16])   // mat.cpp:307-319
{
    float itan = 1 / tanf(radians(fov) * 0.5f);
    float id = 1 / (znear - zfar);
    float r[16] = {itan / aspect, 0, 0, 0,
                   0, itan, 0, 0,
                   0, 0, (zfar + znear) * id, 2.f * zfar * znear * id,
                   0, 0, -1, 0};
    std::memcpy(m, r, sizeof(r));
}

bool inverse(const float in[16], float out[16])   // mat.cpp:378-447 (Gauss-Jordan, full pivoting)
{
    float m[4][4];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) m[i][j] = in[4 * i + j];
    int indxc[4], indxr[4];
    int ipiv[4] = {0, 0, 0, 0};
    bool ok = true;
    for (int i = 0; i < 4; i++) {
        int irow = -1, icol = -1;
        float big = 0.f;
        for (int j = 0; j < 4; j++) {
            if (ipiv[j] != 1) {
                for (int k = 0; k < 4; k++) {
                    if (ipiv[k] == 0) {
                        if (fabsf(m[j][k]) >= big) {
                            big = std::abs(m[j][k]);
                            irow = j;
                            icol = k;
                        }
                    } else if (ipiv[k] > 1)
                        ok = false;
                }
            }
        }
        if (irow < 0 || icol < 0) {
            ok = false;
            break;
        }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < 4; ++k) std::swap(m[irow][k], m[icol][k]);
        indxr[i] = irow;
        indxc[i] = icol;
        if (m[icol][icol] == 0.)
            ok = false;
        float pivinv = 1.f / m[icol][icol];
        m[icol][icol] = 1.f;
        for (int j = 0; j < 4; j++) m[icol][j] *= pivinv;
        for (int j = 0; j < 4; j++) {
            if (j != icol) {
                float save = m[j][icol];
                m[j][icol] = 0;
                for (int k = 0; k < 4; k++) m[j][k] -= m[icol][k] * save;
            }
        }
    }
    if (ok) {
        for (int j = 3; j >= 0; j--) {
            if (indxr[j] != indxc[j])
                for (int k = 0; k < 4; k++) std::swap(m[k][indxr[j]], m[k][indxc[j]]);
        }
    }
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = m[i][j];
    return ok;
}

void transform_points(const float m[16], const float* pts, int64_t n, float* out)
{
    for (int64_t i = 0; i < n; i++) {
        v3 p = xform_point(m, mk(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]));
        out[3 * i] = p.x;
        out[3 * i + 1] = p.y;
        out[3 * i + 2] = p.z;
    }
}

}  // namespace mat

// --------------------------------------------------------------------------
// OBJ / MTL
// --------------------------------------------------------------------------
namespace {

std::string pathname(const std::string& filename)   // files.cpp:68-84 (POSIX branch)
{
    std::string path = filename;
    std::replace(path.begin(), path.end(), '\\', '/');
    size_t slash = path.find_last_of('/');
    if (slash != std::string::npos)
        return path.substr(0, slash + 1);
    return "./";
}

std::string normalize_filename(const std::string& filename)   // files.cpp:89-99
{
    std::string path = filename;
    std::replace(path.begin(), path.end(), '\\', '/');
    return path;
}

struct MtlTable {
    std::vector<std::string> names;
    std::vector<ObjMaterial> mats;
    int default_id = -1;

    int find(const char* name) const   // Materials::find, materials.h:96-107
    {
        if (name == nullptr || name[0] == 0)
            return -1;
        for (int i = 0; i < (int)names.size(); i++)
            if (names[i] == name)
                return i;
        return -1;
    }
    int insert(const ObjMaterial& m, const char* name)   // Materials::insert, materials.h:69-80
    {
        int id = find(name);
        if (id == -1) {
            id = (int)mats.size();
            names.push_back(name);
            mats.push_back(m);
        }
        return id;
    }
    int default_material_index()   // materials.h:145-151: Material(Color(0.8f)), "default"
    {
        if (default_id == -1) {
            ObjMaterial m;
            m.diffuse[0] = m.diffuse[1] = m.diffuse[2] = 0.8f;
            default_id = insert(m, "default");
        }
        return default_id;
    }
};

bool read_mtl(const char* filename, MtlTable& table)   // read_materials_mtl, mesh_io.cpp:213-304
{
    FILE* in = fopen(filename, "rt");
    if (!in)
        return false;
    ObjMaterial* material = nullptr;
    int material_id = -1;
    char tmp[1024];
    char line_buffer[1024];
    bool error = true;
    for (;;) {
        if (!fgets(line_buffer, sizeof(line_buffer), in)) {
            error = false;
            break;
        }
        line_buffer[sizeof(line_buffer) - 1] = 0;
        char* line = line_buffer;
        while (*line && isspace(*line)) line++;
        if (line[0] == 'n') {
            if (sscanf(line, "newmtl %[^\r\n]", tmp) == 1) {
                ObjMaterial black;   // Material(Black()): diffuse 0, ambient_coeff 1
                material_id = table.insert(black, tmp);
            }
        }
        material = material_id >= 0 ? &table.mats[material_id] : nullptr;
        if (material == nullptr)
            continue;
        if (line[0] == 'K') {
            float r, g, b;
            if (sscanf(line, "Kd %f %f %f", &r, &g, &b) == 3) {
                material->diffuse[0] = r; material->diffuse[1] = g; material->diffuse[2] = b;
            } else if (sscanf(line, "Ks %f %f %f", &r, &g, &b) == 3) {
                material->specular[0] = r; material->specular[1] = g; material->specular[2] = b;
            } else if (sscanf(line, "Ke %f %f %f", &r, &g, &b) == 3) {
                material->emission[0] = r; material->emission[1] = g; material->emission[2] = b;
            } else if (sscanf(line, "Ka %f %f %f", &r, &g, &b) == 3) {
                material->ambient[0] = r; material->ambient[1] = g; material->ambient[2] = b;
            }
        } else if (line[0] == 'N') {
            float n;
            if (sscanf(line, "Ns %f", &n) == 1)
                material->ns = n;
            if (sscanf(line, "Ni %f", &n) == 1)
                material->ni = n;
        }
        // Tf / map_* entries do not reach the hot path (transmission, texture file names)
    }
    fclose(in);
    return !error;
}

struct VKey {   // mesh_io.cpp:403-423
    int material, position, texcoord, normal;
    bool operator<(const VKey& b) const
    {
        if (material != b.material) return material < b.material;
        if (position != b.position) return position < b.position;
        if (texcoord != b.texcoord) return texcoord < b.texcoord;
        if (normal != b.normal) return normal < b.normal;
        return false;
    }
};

}  // namespace

bool load_obj(const char* filename, const float xform[16], int mat_offset, ObjData& out, std::string& err)
{
    out = ObjData();
    FILE* in = fopen(filename, "rt");
    if (!in) {
        err = std::string("cannot open '") + filename + "'";
        return false;
    }
    std::vector<v3> wpositions, wtexcoords;
    std::vector<v3> positions, texcoords;
    std::vector<int> indices, material_indices;
    size_t wnormals = 0;
    std::vector<int> wp, wt, wn;
    std::map<VKey, int> remap;
    MtlTable table;
    int material_id = -1;
    char tmp[1024];
    char line_buffer[1024];
    bool error = true;
    for (;;) {
        if (!fgets(line_buffer, sizeof(line_buffer), in)) {
            error = false;
            break;
        }
        line_buffer[sizeof(line_buffer) - 1] = 0;
        char* line = line_buffer;
        while (*line && isspace(*line)) line++;
        if (line[0] == 'v') {
            float x, y, z;
            if (line[1] == ' ') {
                if (sscanf(line, "v %f %f %f", &x, &y, &z) != 3)
                    break;
                wpositions.push_back(mk(x, y, z));
            } else if (line[1] == 'n') {
                if (sscanf(line, "vn %f %f %f", &x, &y, &z) != 3)
                    break;
                wnormals++;
            } else if (line[1] == 't') {
                if (sscanf(line, "vt %f %f", &x, &y) != 2)
                    break;
                wtexcoords.push_back(mk(x, y, 0));
            }
        } else if (line[0] == 'f') {
            wp.clear();
            wt.clear();
            wn.clear();
            int next;
            for (line = line + 1;; line = line + next) {
                wp.push_back(0);
                wt.push_back(0);
                wn.push_back(0);
                next = 0;
                if (sscanf(line, " %d/%d/%d %n", &wp.back(), &wt.back(), &wn.back(), &next) == 3)
                    continue;
                else if (sscanf(line, " %d/%d %n", &wp.back(), &wt.back(), &next) == 2)
                    continue;
                else if (sscanf(line, " %d//%d %n", &wp.back(), &wn.back(), &next) == 2)
                    continue;
                else if (sscanf(line, " %d %n", &wp.back(), &next) == 1)
                    continue;
                else if (next == 0)
                    break;
            }
            if (material_id == -1 && !table.mats.empty())
                material_id = table.default_material_index();
            for (unsigned v = 2; v + 1 < wp.size(); v++) {   // fan triangulation, mesh_io.cpp:524-553
                material_indices.push_back(material_id);
                unsigned idv[3] = {0, v - 1, v};
                for (unsigned i = 0; i < 3; i++) {
                    unsigned k = idv[i];
                    int p = (wp[k] < 0) ? (int)wpositions.size() + wp[k] : wp[k] - 1;
                    int t = (wt[k] < 0) ? (int)wtexcoords.size() + wt[k] : wt[k] - 1;
                    int n = (wn[k] < 0) ? (int)wnormals + wn[k] : wn[k] - 1;
                    if (p < 0)
                        break;
                    auto found = remap.insert(std::make_pair(VKey{material_id, p, t, n}, (int)remap.size()));
                    if (found.second) {
                        if (t != -1) texcoords.push_back(wtexcoords[t]);
                        positions.push_back(wpositions[p]);
                    }
                    indices.push_back(found.first->second);
                }
            }
        } else if (line[0] == 'm') {
            if (sscanf(line, "mtllib %[^\r\n]", tmp) == 1) {
                std::string materials_filename;
                if (tmp[0] != '/' && tmp[1] != ':')
                    materials_filename = normalize_filename(pathname(filename) + tmp);
                else
                    materials_filename = std::string(tmp);
                if (!read_mtl(materials_filename.c_str(), table))
                    break;
            }
        } else if (line[0] == 'u') {
            if (sscanf(line, "usemtl %[^\r\n]", tmp) == 1)
                material_id = table.find(tmp);
        }
    }
    fclose(in);
    if (error) {
        err = std::string("parse error in '") + filename + "'";
        return false;
    }
    // MeshIOUtils::create_triangles (meshIOUtils.cpp:4-30)
    size_t ntri = indices.size() / 3;
    out.tri.resize(ntri * 9);
    out.mat.resize(ntri);
    out.has_uv = !texcoords.empty();
    if (out.has_uv)
        out.uv.resize(ntri * 6);
    for (size_t i = 0; i < ntri; i++) {
        for (int k = 0; k < 3; k++) {
            v3 p = xform_point(xform, positions[indices[3 * i + k]]);
            out.tri[9 * i + 3 * k] = p.x;
            out.tri[9 * i + 3 * k + 1] = p.y;
            out.tri[9 * i + 3 * k + 2] = p.z;
        }
        out.mat[i] = material_indices[i] + mat_offset;
        if (out.has_uv) {
            for (int k = 0; k < 3; k++) {
                // meshData.texcoords[index] (texcoords are only pushed for vertices that have one)
                size_t vi = (size_t)indices[3 * i + k];
                v3 t = vi < texcoords.size() ? texcoords[vi] : mk(0, 0, 0);
                out.uv[6 * i + k] = t.x;
                out.uv[6 * i + 3 + k] = t.y;
            }
        }
    }
    out.materials = table.mats;
    return true;
}

}  // namespace rt
