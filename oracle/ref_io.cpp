// ref_io.cpp -- test infrastructure (the checker, never the product): the reference's own
// vendored OBJ and PNG readers, compiled UNMODIFIED from /root/reference, behind a small C
// interface for tests/test_ref_io.py and tests/golden/make_ref_fixtures.py.
//
//   * template/tiny_obj_loader.h (tinyobjloader, vendored by the reference; compiled with
//     TINYOBJLOADER_IMPLEMENTATION exactly as template/precomp.h:1658-1659 does), called the
//     way Scene::LoadModel calls it (template/scene.h:156-201): LoadObj with its default
//     triangulate = true, then every face's corners through LoadModel's sliding triV window,
//     one triangle per completed window;
//   * lib/stb_image.h (stb_image v2.27, vendored; STB_IMAGE_IMPLEMENTATION with the
//     STBI_NO_PSD / STBI_NO_PIC / STBI_NO_PNM options of template/template.cpp:6-10), called
//     the way Surface::LoadImage does (template/template.cpp:1579-1601): stbi_load with 0
//     requested channels, then 0x00RRGGBB texels (grey: p + p<<8 + p<<16; otherwise the first
//     three channels).
//
// Only the headers are the reference's; this file is the driver.  Built by oracle/Makefile
// (target ref) into oracle/_ref/libref_io.so when /root/reference is present; no stand-in
// header, no edit of the reference sources.  The GPU box has no /root/reference: tests there
// use the committed digests in tests/golden/ref_meshes.json instead.
#define TINYOBJLOADER_IMPLEMENTATION
#include "tiny_obj_loader.h"

#define STB_IMAGE_IMPLEMENTATION
#define STBI_NO_PSD
#define STBI_NO_PIC
#define STBI_NO_PNM
#include "stb_image.h"

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {
template <typename T>
T *copy_out(const std::vector<T> &v) {
    T *p = static_cast<T *>(std::malloc(sizeof(T) * (v.empty() ? 1 : v.size())));
    if (p && !v.empty()) std::memcpy(p, v.data(), sizeof(T) * v.size());
    return p;
}
}  // namespace

extern "C" {

// tinyobj::LoadObj(path) as Scene::LoadModel runs it.  Outputs (malloc'd, free with ref_free):
//   verts[3 * nv]  attrib.vertices (the parsed floats, file order)
//   corners[3 * nt] the vertex_index of each triangle corner, in the order LoadModel creates
//                   the triangles (shapes, then faces, then the triV window)
// Returns 0, or -1 when LoadObj fails (LoadModel prints and returns without triangles).
int ref_load_model(const char *path, float **verts, uint32_t *nv, int32_t **corners, uint32_t *nt) {
    tinyobj::attrib_t attrib;
    std::vector<tinyobj::shape_t> shapes;
    std::vector<tinyobj::material_t> materials;
    std::string warn, err;
    if (!tinyobj::LoadObj(&attrib, &shapes, &materials, &warn, &err, path)) return -1;
    std::vector<int32_t> tri;
    for (size_t s = 0; s < shapes.size(); ++s) {
        size_t index_offset = 0;
        for (size_t f = 0; f < shapes[s].mesh.num_face_vertices.size(); ++f) {
            const size_t fv = shapes[s].mesh.num_face_vertices[f];
            std::vector<int32_t> window;   // LoadModel's triV, as vertex indices
            for (size_t v = 0; v < fv; ++v) {
                window.push_back(shapes[s].mesh.indices[index_offset + v].vertex_index);
                if (window.size() == 3) {
                    tri.insert(tri.end(), window.begin(), window.end());
                    window.erase(window.begin());
                }
            }
            index_offset += fv;
        }
    }
    std::vector<float> v(attrib.vertices.begin(), attrib.vertices.end());
    *verts = copy_out(v);
    *nv = (uint32_t)(v.size() / 3);
    *corners = copy_out(tri);
    *nt = (uint32_t)(tri.size() / 3);
    return 0;
}

// stbi_load(path, 0 channels) + Surface::LoadImage's texel packing.  pixels (malloc'd) =
// 0x00RRGGBB, row-major; *channels = stb's channel count n.  Returns 0, -1 if stb fails.
int ref_load_image(const char *path, uint32_t **pixels, int *width, int *height, int *channels) {
    int w = 0, h = 0, n = 0;
    unsigned char *data = stbi_load(path, &w, &h, &n, 0);
    if (!data) return -1;
    const size_t s = (size_t)w * h;
    uint32_t *p = static_cast<uint32_t *>(std::malloc(sizeof(uint32_t) * (s ? s : 1)));
    if (!p) { stbi_image_free(data); return -1; }
    if (n == 1) {
        for (size_t i = 0; i < s; ++i) {
            const unsigned char g = data[i];
            p[i] = g + (g << 8) + (g << 16);
        }
    } else {
        for (size_t i = 0; i < s; ++i)
            p[i] = ((uint32_t)data[i * n + 0] << 16) + ((uint32_t)data[i * n + 1] << 8) + data[i * n + 2];
    }
    stbi_image_free(data);
    *pixels = p;
    *width = w;
    *height = h;
    *channels = n;
    return 0;
}

void ref_free(void *p) { std::free(p); }

}  // extern "C"
