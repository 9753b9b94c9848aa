/* render_golden.c -- a plain C caller of include/rt_mi355x.h, the way a reference-side adapter
 *  drives the library: settings, camera, light, materials and triangles from a
 * scene file written by tests/test_c_api.py, then rt_render (render(Renderer&), mainUtils.cpp:6-21)
 * and rt_get_image (Renderer::get_image, renderer.cpp:106-109).
 *
 *   render_golden SCENE OUT [DEVICES...]
 *
 * With device ids after OUT, rt_set_devices(ids) comes before the render (ids[0] = 0).
 * OUT receives int32 width, int32 height, then width x height ARGB32 words.
 * Scene file (little endian): "RTSC", int32 sizeof(rt_settings), rt_settings, float cam_pos[3],
 * proj_inv[16], cam_to_world[16], int32 has_proj, proj[16], world_to_cam[16], float fov, aspect,
 * light[3], int32 nmat, float mats[nmat][16], int64 ntri, float tri9[ntri][9], int32 mat[ntri],
 * int32 has_uv, float uv6[ntri][6] (when has_uv). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_mi355x.h"

static int read_all(FILE *f, void *p, size_t n)
{
    return fread(p, 1, n, f) == n;
}

static void *read_array(FILE *f, size_t n)
{
    void *p = malloc(n ? n : 1);
    if (p && !read_all(f, p, n)) {
        free(p);
        return NULL;
    }
    return p;
}

#define CHECK(call)                                                                   \
    do {                                                                              \
        int rc_ = (call);                                                             \
        if (rc_ != RT_OK) {                                                           \
            fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, rt_last_error());     \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

int main(int argc, char **argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s SCENE OUT [DEVICES...]\n", argv[0]);
        return 2;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) {
        perror(argv[1]);
        return 2;
    }
    char magic[4];
    int32_t settings_size, has_proj, nmat, has_uv;
    rt_settings st;
    float cam_pos[3], proj_inv[16], c2w[16], proj[16], w2c[16], fov, aspect, light[3];
    int64_t ntri;
    if (!read_all(f, magic, 4) || memcmp(magic, "RTSC", 4) || !read_all(f, &settings_size, 4) ||
        settings_size != (int32_t)sizeof(rt_settings) || !read_all(f, &st, sizeof st) || !read_all(f, cam_pos, 12) ||
        !read_all(f, proj_inv, 64) || !read_all(f, c2w, 64) || !read_all(f, &has_proj, 4) || !read_all(f, proj, 64) ||
        !read_all(f, w2c, 64) || !read_all(f, &fov, 4) || !read_all(f, &aspect, 4) || !read_all(f, light, 12) ||
        !read_all(f, &nmat, 4)) {
        fprintf(stderr, "bad scene header (rt_settings is %zu bytes here)\n", sizeof(rt_settings));
        return 2;
    }
    float *mats = read_array(f, (size_t)nmat * 16 * sizeof(float));
    if (!mats || !read_all(f, &ntri, 8))
        return 2;
    float *tri9 = read_array(f, (size_t)ntri * 9 * sizeof(float));
    int32_t *mat = read_array(f, (size_t)ntri * sizeof(int32_t));
    if (!tri9 || !mat || !read_all(f, &has_uv, 4))
        return 2;
    float *uv6 = has_uv ? read_array(f, (size_t)ntri * 6 * sizeof(float)) : NULL;
    if (has_uv && !uv6)
        return 2;
    fclose(f);

    rt_renderer *r = rt_create(0);
    if (!r) {
        fprintf(stderr, "rt_create: %s\n", rt_last_error());
        return 1;
    }
    CHECK(rt_set_settings(r, &st));
    CHECK(rt_change_render_size(r, st.image_width, st.image_height));
    CHECK(rt_set_camera_matrices(r, cam_pos, proj_inv, c2w));
    if (has_proj)
        CHECK(rt_set_camera_projection(r, proj, w2c));
    CHECK(rt_set_camera_lens(r, fov, aspect));
    CHECK(rt_set_light_position(r, light[0], light[1], light[2]));
    CHECK(rt_set_materials(r, mats, nmat));
    CHECK(rt_clear_geometry(r));
    CHECK(rt_set_triangles(r, tri9, mat, uv6, ntri));
    if (argc > 3) {
        int32_t ids[16];
        int32_t n = 0;
        for (int i = 3; i < argc && n < 16; i++)
            ids[n++] = (int32_t)atoi(argv[i]);
        CHECK(rt_set_devices(r, ids, n));
    }
    float ms = 0.0f;
    CHECK(rt_render(r, &ms));
    int32_t w = 0, h = 0;
    CHECK(rt_get_image(r, NULL, &w, &h));
    uint32_t *img = malloc((size_t)w * h * sizeof(uint32_t));
    if (!img)
        return 1;
    CHECK(rt_get_image(r, img, &w, &h));
    FILE *o = fopen(argv[2], "wb");
    if (!o || fwrite(&w, 4, 1, o) != 1 || fwrite(&h, 4, 1, o) != 1 ||
        fwrite(img, sizeof(uint32_t), (size_t)w * h, o) != (size_t)w * h) {
        perror(argv[2]);
        return 1;
    }
    fclose(o);
    printf("rendered %dx%d in %.2f ms\n", w, h, ms);
    rt_destroy(r);
    free(img);
    free(mats);
    free(tri9);
    free(mat);
    free(uv6);
    return 0;
}
