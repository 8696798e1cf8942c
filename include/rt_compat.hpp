// rt_compat.hpp -- header-only C++ shim keeping the reference's class surface on top of
// the librtamd.so C-ABI, so a host written against pmichels19/AdvancedGraphicsRayTracer's
// Renderer / Scene / Camera / Ray (renderer.h, template/scene.h, camera.h, Ray.h) can
// switch to the MI355X path by swapping includes.
//
//   Tmpl8::Ray                 Ray.h:7-32 (O, D, rD, t, objIdx, inside, u, v)
//   Tmpl8::Scene::IntersectBVH template/scene.h:285   -> rt_intersect_host (batch of 1 or n)
//   Tmpl8::Scene::IsOccluded   template/scene.h:452   -> rt_occluded_host
//   Tmpl8::Scene::IntersectBVHPacket template/scene.h:322 -> rt_intersect_packets_host
//   Tmpl8::Camera              camera.h:28-52         -> rt_camera_default
//   Tmpl8::Renderer::Tick      renderer.cpp:200-309   -> rt_render_frame_host
//   Tmpl8::Renderer::Trace     renderer.cpp:17-72     -> rt_trace_host (WhittedTrace: 138-195)
//
// Per-ray calls cross PCIe; batch them (the vector overloads) for throughput.  There is
// no CPU fallback: every call reports the library's error through RtError.
#pragma once
#include <stdexcept>
#include <string>
#include <vector>

#include "rt_amd.h"

namespace Tmpl8 {

struct RtError : std::runtime_error {
    int code;
    RtError(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};
inline void rt_check(int rc) {
    if (rc != RT_OK) throw RtError(rc, rt_last_error());
}

struct float3 { float x = 0, y = 0, z = 0; };

class Ray {   // Ray.h:7-32
  public:
    Ray() = default;
    Ray(float3 origin, float3 direction, float distance = 1e34f) : O(origin), D(direction), t(distance) {
        rD = float3{1 / D.x, 1 / D.y, 1 / D.z};
    }
    float3 IntersectionPoint() const { return float3{O.x + t * D.x, O.y + t * D.y, O.z + t * D.z}; }
    float3 O, D, rD;
    float t = 1e34f;
    int objIdx = -1;
    bool inside = false;
    float u = 0, v = 0;
};

constexpr int PACKET_SIZE = 64;   // Ray.h:4

struct RayPacket {   // Ray.h:34-64 (SoA, one 8x8 tile of primary rays)
    float3 O[PACKET_SIZE], D[PACKET_SIZE];
    float t[PACKET_SIZE], u[PACKET_SIZE] = {}, v[PACKET_SIZE] = {};
    int objIdx[PACKET_SIZE];
    int firstActive = 0;
    RayPacket() {
        for (int i = 0; i < PACKET_SIZE; ++i) t[i] = 1e34f, objIdx[i] = -1;
    }
};

class Scene {   // template/scene.h:37
  public:
    explicit Scene(const char *recipe, const char *mesh_dir, int device = 0) {
        rt_check(rt_scene_create_recipe(recipe, mesh_dir, device, &h_));
    }
    explicit Scene(const rt_scene_desc &desc) { rt_check(rt_scene_create(&desc, &h_)); }
    Scene(const Scene &) = delete;
    Scene &operator=(const Scene &) = delete;
    ~Scene() { rt_scene_destroy(h_); }

    void IntersectBVH(Ray &ray) { std::vector<Ray *> one{&ray}; IntersectBVH(one); }
    bool IsOccluded(Ray &ray) { std::vector<Ray *> one{&ray}; return IsOccluded(one)[0]; }

    void IntersectBVH(std::vector<Ray *> &rays) {
        std::vector<rt_ray> in = pack(rays);
        std::vector<rt_hit> out(in.size());
        rt_check(rt_intersect_host(h_, in.data(), out.data(), (uint32_t)in.size()));
        for (size_t i = 0; i < rays.size(); ++i) {
            if (out[i].obj < 0) continue;   // nothing closer than ray.t: the ray is left as it was
            rays[i]->t = out[i].t;
            rays[i]->objIdx = out[i].obj;
            rays[i]->u = out[i].u;
            rays[i]->v = out[i].v;
        }
    }
    // Scene::IntersectBVHPacket (template/scene.h:322-412) on one or more packets
    void IntersectBVHPacket(RayPacket &p) { IntersectBVHPacket(&p, 1); }
    void IntersectBVHPacket(RayPacket *packets, size_t count) {
        std::vector<rt_ray> in(count * PACKET_SIZE);
        for (size_t k = 0; k < count; ++k)
            for (int i = 0; i < PACKET_SIZE; ++i) {
                const RayPacket &p = packets[k];
                in[k * PACKET_SIZE + i] = rt_ray{p.O[i].x, p.O[i].y, p.O[i].z, p.D[i].x, p.D[i].y, p.D[i].z, p.t[i]};
            }
        std::vector<rt_hit> out(in.size());
        rt_check(rt_intersect_packets_host(h_, in.data(), out.data(), (uint32_t)in.size()));
        for (size_t k = 0; k < count; ++k)
            for (int i = 0; i < PACKET_SIZE; ++i) {
                const rt_hit &h = out[k * PACKET_SIZE + i];
                if (h.obj < 0) continue;
                packets[k].t[i] = h.t; packets[k].objIdx[i] = h.obj; packets[k].u[i] = h.u; packets[k].v[i] = h.v;
            }
    }
    std::vector<bool> IsOccluded(std::vector<Ray *> &rays) {
        std::vector<rt_ray> in = pack(rays);
        std::vector<uint8_t> out(in.size());
        rt_check(rt_occluded_host(h_, in.data(), out.data(), (uint32_t)in.size()));
        return std::vector<bool>(out.begin(), out.end());
    }
    rt_scene_info Info() const { rt_scene_info i{}; rt_check(rt_scene_get_info(h_, &i)); return i; }
    rt_scene *handle() const { return h_; }

  private:
    rt_scene *h_ = nullptr;
    static std::vector<rt_ray> pack(const std::vector<Ray *> &rays) {
        std::vector<rt_ray> in(rays.size());
        for (size_t i = 0; i < rays.size(); ++i) {
            const Ray &r = *rays[i];
            in[i] = rt_ray{r.O.x, r.O.y, r.O.z, r.D.x, r.D.y, r.D.z, r.t};
        }
        return in;
    }
};

class Camera {   // camera.h:28-41
  public:
    Camera(uint32_t width, uint32_t height) { rt_check(rt_camera_default(width, height, &cam)); }
    rt_camera cam{};
};

class Renderer {   // renderer.h:5-160
  public:
    Renderer(Scene &scene, uint32_t width, uint32_t height)
        : scene(scene), camera(width, height), width_(width), height_(height), pixels(size_t(width) * height) {
        rt_check(rt_renderer_create(scene.handle(), width, height, &h_));
    }
    Renderer(const Renderer &) = delete;
    Renderer &operator=(const Renderer &) = delete;
    ~Renderer() { rt_renderer_destroy(h_); }

    // One frame: Trace (depth 10, renderer.h:9) or WhittedTrace (depth 20, renderer.h:13)
    // per pixel, accumulate, pack into pixels.  depth 0 = the reference's default.
    // usePackets = the PACKET_TRAVERSAL build (Ray.h:3): 8x8 packets through TracePacket.
    void Tick(float /*deltaTime*/, uint32_t depth = 0, uint32_t spp = 1) {
        if (depth == 0) depth = useWhitted ? 20 : 10;
        const uint32_t mode = useWhitted ? RT_MODE_WHITTED : usePackets ? RT_MODE_PACKET : RT_MODE_PATH;
        rt_frame_params p{width_, height_, spp, depth, frame_++, mode, swapped_ ? 1u : 0u};
        swapped_ = false;
        rt_check(rt_render_frame_host(h_, &camera.cam, &p, pixels.data()));
    }
    // Renderer::Trace (renderer.h:9, renderer.cpp:17-72) and WhittedTrace (renderer.h:13,
    // renderer.cpp:138-195) on one ray: the reference's RandomFloat() advances one global seed
    // (template/template.cpp:673-686); `seed` plays that role and advances the same way.  As
    // Trace takes Ray&, the ray is left as the first IntersectBVH leaves it (renderer.cpp:20).
    float3 Trace(Ray &ray, bool lastSpecular = true, int depth = 10) {
        std::vector<Ray *> one{&ray};
        std::vector<uint32_t> seeds{seed};
        float3 c = Trace(one, seeds, lastSpecular, depth)[0];
        seed = seeds[0];
        return c;
    }
    float3 WhittedTrace(Ray &ray, int depth = 20) {
        std::vector<Ray *> one{&ray};
        std::vector<uint32_t> seeds{seed};
        float3 c = run_trace(RT_MODE_WHITTED, one, seeds, true, depth)[0];
        seed = seeds[0];
        return c;
    }
    // Batched Trace: ray i draws from seeds[i] (updated in place); one launch for the batch.
    std::vector<float3> Trace(std::vector<Ray *> &rays, std::vector<uint32_t> &seeds, bool lastSpecular = true,
                              int depth = 10) {
        return run_trace(RT_MODE_PATH, rays, seeds, lastSpecular, depth);
    }
    uint32_t seed = 0x12345678;     // template/template.cpp:673

    // The K key (renderer.h:138): switch integrators; the next frame restarts accumulation.
    void ToggleWhitted() { useWhitted = !useWhitted; swapped_ = true; }
    rt_counters Counters() { rt_counters c{}; rt_check(rt_renderer_counters(h_, &c)); return c; }

    Scene &scene;
    Camera camera;

  private:
    std::vector<float3> run_trace(int mode, std::vector<Ray *> &rays, std::vector<uint32_t> &seeds, bool lastSpecular,
                                  int depth) {
        if (seeds.size() != rays.size() || depth < 0) throw RtError(RT_ERR_INVALID, "Trace: one seed per ray");
        std::vector<rt_ray> in(rays.size());
        std::vector<uint8_t> flags(rays.size());
        for (size_t i = 0; i < rays.size(); ++i) {
            const Ray &r = *rays[i];
            in[i] = rt_ray{r.O.x, r.O.y, r.O.z, r.D.x, r.D.y, r.D.z, r.t};
            flags[i] = (uint8_t)((lastSpecular ? 1 : 0) | (r.inside ? 2 : 0));
        }
        std::vector<float> rad(3 * rays.size());
        std::vector<rt_hit> hits(rays.size());
        rt_check(rt_trace_host(scene.handle(), mode, in.data(), seeds.data(), flags.data(), (uint32_t)depth, rad.data(),
                               hits.data(), nullptr, (uint32_t)in.size()));
        std::vector<float3> out(rays.size());
        for (size_t i = 0; i < rays.size(); ++i) {
            out[i] = float3{rad[3 * i], rad[3 * i + 1], rad[3 * i + 2]};
            if (hits[i].obj >= 0) {
                rays[i]->t = hits[i].t; rays[i]->objIdx = hits[i].obj; rays[i]->u = hits[i].u; rays[i]->v = hits[i].v;
            }
        }
        return out;
    }
    uint32_t width_, height_;
    uint32_t frame_ = 0;
    bool swapped_ = false;
    rt_renderer *h_ = nullptr;

  public:
    bool useWhitted = false;        // renderer.h:158
    bool usePackets = false;        // PACKET_TRAVERSAL, Ray.h:3
    std::vector<uint32_t> pixels;   // 0x00RRGGBB, the reference's screen->pixels
};

}  // namespace Tmpl8
