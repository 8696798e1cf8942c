// rt_internal.h -- host-side internals shared by rt_host.cpp and rt_device.hip.
#pragma once
#include <string>
#include <vector>

#include "../../include/rt_amd.h"
#include "rt_math.h"

namespace rt {

// thread-local error message for rt_last_error()
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

// 32-byte BVHNode (BVHNode.h:5-14): aabbMin, aabbMax, leftFirst, primitiveCount
struct Node {
    float mn[3], mx[3];
    uint32_t leftFirst, count;
};
static_assert(sizeof(Node) == 32, "BVHNode layout");

// Primitive::Transform and InvertedTransform (Primitive.h:28-29, 39-41): Translate(centre)
// for spheres, T * Translate(pos) (|pos| > FLT_EPSILON) or T for cubes, T for quads,
// identity otherwise.  T16 = the caller's mat4 (NULL = identity).
struct PrimX { float M[16], Minv[16]; };
void prim_transform(const rt_prim &p, const float *T16, PrimX &x);
// mat4::FastInvertedTransformNoScale (template/precomp.h:1061-1085)
void fast_inverse(const float *M, float *out);

// Per-primitive geometry the builder and the uploader need, evaluated exactly as
// Primitive::GetCentroid / GetAABBMin / GetAABBMax (Primitive.h:42-50, 319-388, 443-445).
struct PrimGeom { f3 centroid, bmin, bmax; };
void prim_geometry(const rt_prim &p, const PrimX &x, PrimGeom &g);
void translate_matrix(float x, float y, float z, float M[16]);

// Plain binned-SAH BVH (template/scene.h:845-976).  nodes sized 2N+2, indices N.
struct Bvh {
    std::vector<Node> nodes;
    std::vector<uint32_t> indices;
    uint32_t nodes_used = 0, depth = 0, max_leaf = 0;
};
int build_bvh(const rt_prim *prims, const float *transforms, uint32_t n, Bvh &out);
// Spatial-split BVH (rt_sbvh.cpp): indices hold references (a primitive may repeat)
int build_sbvh(const rt_prim *prims, const float *transforms, uint32_t n, Bvh &out);

// frame size and device of a renderer (rt_multi.cpp)
int renderer_geometry(const rt_renderer *r, uint32_t *W, uint32_t *H, int *device);
// the 8x8 tiles whose running averages the renderer's accumulator holds (its last frame's tiles:
// all of them after a whole frame, a shard's after a shard); false before its first frame
bool renderer_held_tiles(const rt_renderer *r, std::vector<uint32_t> &tiles);
// the renderer's device accumulator (W*H float4 = 16 B each); and the accumulator values of
// the 8x8 tiles listed in DEVICE memory (tiles_dev) packed as [i][64] float4 into buf_dev /
// written back from it (pixels outside the frame: 0 / skipped), in stream order on `stream`
// with no host synchronisation -- rt_multi.cpp moves a pixel's running average to its new rank
// when a multi-GPU deal changes owners
int renderer_accumulator(rt_renderer *r, void **acc_dev, size_t *bytes);
int accumulator_pack(rt_renderer *r, const uint32_t *tiles_dev, uint32_t n, void *buf_dev, void *stream);
int accumulator_unpack(rt_renderer *r, const uint32_t *tiles_dev, uint32_t n, const void *buf_dev, void *stream);
// one rank's part of a multi-GPU frame (rt_multi.cpp): the interleaved shard `shard` of
// `nshards`, or the explicit tile list `tiles` (n tiles; n == 0 with tiles != NULL: none),
// written packed ([local tile][64], rt_render_shard's layout) or, packed == 0, straight into a
// row-major W x H frame at the tiles' own pixels (rank 0 renders its tiles into the output frame).
// fwd_src / fwd_dst (row-major only, may be NULL): as each pixel is stored, its value in fwd_src is
// first forwarded to fwd_dst (the previous frame handed to the caller within the same launch)
int render_part(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t shard, uint32_t nshards,
                const uint32_t *tiles, uint32_t n, int packed, uint32_t *out_dev, void *stream,
                const uint32_t *fwd_src = nullptr, uint32_t *fwd_dst = nullptr);

// the dry-run work map of the same part of a frame (rt_renderer_tile_work): per local tile, node
// visits + primitive tests summed over its lanes and samples -- deterministic, the multi-GPU
// deals' cost input.  Blocks on `stream`.  RT_ERR_UNSUPPORTED for modes other than RT_MODE_PATH.
int render_work(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t shard, uint32_t nshards,
                const uint32_t *tiles, uint32_t n, std::vector<uint32_t> &work, void *stream);

// SURVEY.md 8(d) scenes as descriptions
struct SceneSource {
    std::vector<rt_prim> prims;
    std::vector<rt_material> materials;
};
int recipe_source(const std::string &name, const std::string &mesh_dir, SceneSource &out);

}  // namespace rt
