/*
 * abi_smoke.c -- a plain C caller of include/bih.h (test infrastructure).
 *
 * What the reference's host code would do through the C ABI in place of
 * Renderer::Render (src/Renderer.cpp:415) -> Launch_cudaRender
 * (src/CUDAKernels.cu:425-447): build the BIH of a triangle soup, take the
 * reference camera, render a frame into a host framebuffer, render a row tile,
 * and check every error path it can reach without a device.
 *
 *   abi_smoke --errors                       error codes only (no device)
 *   abi_smoke SCENE.f32 N W H FRAME GOLDEN.u32
 *       SCENE.f32  N*9 float32 (file order), GOLDEN.u32 W*H uint32 0x00BBGGRR
 *
 * Exit 0 = every check passed; prints one line per check.  Built by
 * tests/test_c_abi.py with gcc -std=c11 -Wall -Werror against
 * -lbih_amd (no C++ and no HIP headers on this side of the boundary).
 */
#include "bih.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int g_fail = 0;

#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (cond) {                                        \
            printf("ok   ");                               \
        } else {                                           \
            printf("FAIL ");                               \
            g_fail = 1;                                    \
        }                                                  \
        printf(__VA_ARGS__);                               \
        printf("\n");                                      \
    } while (0)

static void *read_file(const char *path, size_t bytes) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    void *p = malloc(bytes ? bytes : 1);
    size_t got = p ? fread(p, 1, bytes, f) : 0;
    fclose(f);
    if (got != bytes) { free(p); return NULL; }
    return p;
}

static void check_errors(void) {
    bih_tree *t = NULL;
    bih_camera cam;
    CHECK(bih_abi_version() == BIH_ABI_VERSION, "abi version %d", bih_abi_version());
    CHECK(bih_strerror(BIH_ERR_NO_DEVICE) != NULL && bih_strerror(12345) != NULL, "strerror");
    CHECK(bih_build(NULL, 0, &t) == BIH_ERR_INVALID, "bih_build(NULL) -> BIH_ERR_INVALID");
    bih_scene big = {BIH_MAX_TRIS + 1u, (const float *)&big};
    CHECK(bih_build(&big, 0, &t) == BIH_ERR_TOO_LARGE, "oversize scene -> BIH_ERR_TOO_LARGE");
    CHECK(bih_camera_reference(0, 480, &cam) == BIH_ERR_INVALID, "zero-width camera -> INVALID");
    CHECK(bih_render(NULL, NULL, NULL, NULL) == BIH_ERR_INVALID, "bih_render(NULL) -> INVALID");
    CHECK(bih_camera_reference(640, 480, &cam) == BIH_OK && cam.origin[0] == 2.0f &&
              cam.origin[2] == -2.0f && cam.lower_left[1] == -1.0f,
          "reference camera (Renderer.cpp:99, Camera.cu:5-9)");
    bih_scene bad;
    uint32_t line = 0;
    CHECK(bih_scene_load_obj("/nonexistent/x.obj", &bad, &line) == BIH_ERR_IO, "missing OBJ -> IO");
    CHECK(bih_host_register(NULL, 16) == BIH_ERR_INVALID && bih_host_unregister(NULL) == BIH_ERR_INVALID,
          "bih_host_register(NULL) -> INVALID");
    double hist[3];
    CHECK(bih_render_history(NULL, 1, hist) == BIH_ERR_INVALID, "bih_render_history(NULL) -> INVALID");
}

int main(int argc, char **argv) {
    check_errors();
    if (argc == 2 && !strcmp(argv[1], "--errors")) return g_fail;
    if (argc != 7) {
        fprintf(stderr, "usage: abi_smoke SCENE.f32 N W H FRAME GOLDEN.u32 | --errors\n");
        return 2;
    }
    uint32_t n = (uint32_t)strtoul(argv[2], NULL, 10);
    uint32_t w = (uint32_t)strtoul(argv[3], NULL, 10);
    uint32_t h = (uint32_t)strtoul(argv[4], NULL, 10);
    uint32_t frame = (uint32_t)strtoul(argv[5], NULL, 10);
    float *v = (float *)read_file(argv[1], (size_t)n * 9 * sizeof(float));
    uint32_t *golden = (uint32_t *)read_file(argv[6], (size_t)w * h * 4);
    if (!v || !golden) { fprintf(stderr, "cannot read inputs\n"); return 2; }
    CHECK(bih_device_count() > 0, "device count %d", bih_device_count());
    if (g_fail) return 1;

    bih_scene scene = {n, v};
    bih_tree *tree = NULL;
    int rc = bih_build(&scene, 0, &tree);
    CHECK(rc == BIH_OK && tree, "bih_build: %s", bih_strerror(rc));
    if (rc) return 1;
    bih_tree_info info;
    rc = bih_tree_get_info(tree, &info);
    CHECK(rc == BIH_OK && info.n_tris == n && info.n_unique > 0 && info.n_unique <= n,
          "tree info: N=%u U=%u", info.n_tris, info.n_unique);
    bih_camera cam;
    bih_camera_reference(w, h, &cam);

    /* the reference's first frames on one persistent RNG state, up to FRAME */
    uint32_t *img = (uint32_t *)calloc((size_t)w * h, 4);
    for (uint32_t f = 0; f <= frame; ++f) {
        bih_framebuffer fb = {w, h, 4, f, 1984u, img};
        rc = bih_render(&scene, tree, &cam, &fb);
        if (rc) break;
    }
    CHECK(rc == BIH_OK, "bih_render frames 0..%u: %s", frame, bih_strerror(rc));
    size_t diff = 0;
    for (size_t i = 0; i < (size_t)w * h; ++i) diff += img[i] != golden[i];
    CHECK(diff == 0, "frame %u vs golden: %zu of %u pixels differ", frame, diff, w * h);

    /* a row tile of the same frame through bih_render_rows (global pixel RNG) */
    uint32_t r0 = h / 3, nr = h / 4 ? h / 4 : 1;
    uint32_t *tile = (uint32_t *)calloc((size_t)w * nr, 4);
    bih_framebuffer fbt = {w, h, 4, frame, 1984u, tile};
    rc = bih_render_rows(&scene, tree, &cam, &fbt, r0, nr);
    CHECK(rc == BIH_OK && !memcmp(tile, golden + (size_t)r0 * w, (size_t)w * nr * 4),
          "bih_render_rows rows [%u, %u) equal the golden rows: %s", r0, r0 + nr, bih_strerror(rc));

    /* the reference rebuilds every frame: a rebuild leaves the frame unchanged */
    rc = bih_rebuild(tree);
    memset(img, 0, (size_t)w * h * 4);
    bih_framebuffer fb2 = {w, h, 4, frame, 1984u, img};
    int rc2 = bih_render(&scene, tree, &cam, &fb2);
    CHECK(rc == BIH_OK && rc2 == BIH_OK && !memcmp(img, golden, (size_t)w * h * 4),
          "bih_rebuild + bih_render(frame %u) equals golden", frame);

    /* INTEGRATION.md's frame loop into a page-locked framebuffer: rebuild +
       render, several frames, the frame of the golden last */
    rc = bih_host_register(img, (size_t)w * h * 4);
    CHECK(rc == BIH_OK, "bih_host_register: %s", bih_strerror(rc));
    for (uint32_t f = (frame >= 3 ? frame - 3 : 0); f <= frame && rc == BIH_OK; ++f) {
        rc = bih_rebuild(tree);
        bih_framebuffer fl = {w, h, 4, f, 1984u, img};
        if (rc == BIH_OK) rc = bih_render(&scene, tree, &cam, &fl);
    }
    CHECK(rc == BIH_OK && !memcmp(img, golden, (size_t)w * h * 4),
          "rebuild + render loop into a registered framebuffer ends on the golden frame: %s", bih_strerror(rc));
    CHECK(bih_host_unregister(img) == BIH_OK, "bih_host_unregister");

    /* errors that need a tree */
    bih_framebuffer bad = {w, h, 0, 0, 1984u, img};
    CHECK(bih_render(&scene, tree, &cam, &bad) == BIH_ERR_INVALID, "spp 0 -> BIH_ERR_INVALID");
    bih_scene other = {n > 1 ? n - 1 : 2, v};
    CHECK(bih_render(&other, tree, &cam, &fb2) == BIH_ERR_MISMATCH, "foreign scene -> MISMATCH");
    bih_free(tree);
    free(tile); free(img); free(v); free(golden);
    printf("%s\n", g_fail ? "abi_smoke FAILED" : "abi_smoke OK");
    return g_fail;
}
