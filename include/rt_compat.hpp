// rt_compat.hpp -- header-only C++ shim keeping the reference's class surface on top of
// the librtamd.so C-ABI, so a host written against pmichels19/AdvancedGraphicsRayTracer's
// Renderer / Scene / Camera / Ray / Surface / TheApp (renderer.h, template/scene.h, camera.h,
// Ray.h, template/precomp.h) can switch to the MI355X path by swapping includes.
//
//   Tmpl8::float3 / float4     template/precomp.h:255-272 + the float3 operators and helpers
//                              of 533-855 (component-wise, normalize = v * (1/sqrtf(dot)))
//   Tmpl8::Surface             template/precomp.h:110-135, Surface(file) = LoadImage (PNG)
//   Tmpl8::TheApp              template/precomp.h:1640-1654 (the host's app pointer type)
//   Tmpl8::Ray                 Ray.h:7-32 (O, D, rD, t, objIdx, inside, u, v)
//   Tmpl8::Scene()             template/scene.h:40-128: the reference's default scene
//   Tmpl8::Scene::IntersectBVH template/scene.h:285   -> rt_intersect_host (batch of 1 or n)
//   Tmpl8::Scene::IsOccluded   template/scene.h:452   -> rt_occluded_host
//   Tmpl8::Scene::IntersectBVHPacket template/scene.h:322 -> rt_intersect_packets_host
//   Tmpl8::Camera              camera.h:28-52         -> rt_camera_default
//   Tmpl8::Renderer::Init      renderer.cpp:6-12      -> rt_renderer_create (screen size)
//   Tmpl8::Renderer::Tick      renderer.cpp:200-309   -> rt_render_frame_host into screen->pixels
//   Tmpl8::Renderer::Trace     renderer.cpp:17-72     -> rt_trace_host (WhittedTrace: 138-195)
//
// A reference-shaped main (template/template.cpp:133-139, 273, 287) runs unchanged:
//   Surface *screen = new Surface(SCRWIDTH, SCRHEIGHT); Surface *skydome = new Surface(file);
//   TheApp *app = new Renderer(); app->screen = screen; app->skydome = skydome; app->Init();
//   while (...) app->Tick(deltaTime);  app->Shutdown();
// Renderer() builds the reference's default scene (recipe "default": the light, glider and
// mig29 of template/scene.h:80-95 -- the other models it names are not in its assets/) from
// $RT_MESH_DIR (default "assets", the reference's relative paths; *.obj or *.rtmesh), with the
// skydome set before Init() as the sky.  Per-ray calls cross PCIe; batch them (the vector
// overloads) for throughput.  There is no CPU fallback: every call reports the library's error
// through RtError.
#pragma once
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "rt_amd.h"

#ifndef SCRWIDTH
#define SCRWIDTH 1280   // camera.h:4-5
#define SCRHEIGHT 720
#endif

namespace Tmpl8 {

typedef unsigned int uint;

struct RtError : std::runtime_error {
    int code;
    RtError(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};
inline void rt_check(int rc) {
    if (rc != RT_OK) throw RtError(rc, rt_last_error());
}

// ---- vector math, template/precomp.h (the float3 subset the reference's host code uses)
struct float3 {
    float3() = default;
    float3(const float a, const float b, const float c) : x(a), y(b), z(c) {}
    float3(const float a) : x(a), y(a), z(a) {}
    float &operator[](const int n) { return (&x)[n]; }
    float operator[](const int n) const { return (&x)[n]; }
    float x = 0, y = 0, z = 0;
};
struct float4 {
    float4() = default;
    float4(const float a, const float b, const float c, const float d) : x(a), y(b), z(c), w(d) {}
    float4(const float a) : x(a), y(a), z(a), w(a) {}
    float4(const float3 &a, const float d) : x(a.x), y(a.y), z(a.z), w(d) {}
    float x = 0, y = 0, z = 0, w = 0;
};
inline float3 make_float3(const float a, const float b, const float c) { return float3(a, b, c); }
inline float3 make_float3(const float s) { return float3(s, s, s); }
inline float3 operator-(const float3 &a) { return float3(-a.x, -a.y, -a.z); }
inline float3 operator+(const float3 &a, const float3 &b) { return float3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline float3 operator+(const float3 &a, float b) { return float3(a.x + b, a.y + b, a.z + b); }
inline float3 operator+(float b, const float3 &a) { return float3(a.x + b, a.y + b, a.z + b); }
inline void operator+=(float3 &a, const float3 &b) { a.x += b.x; a.y += b.y; a.z += b.z; }
inline void operator+=(float3 &a, float b) { a.x += b; a.y += b; a.z += b; }
inline float3 operator-(const float3 &a, const float3 &b) { return float3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline float3 operator-(const float3 &a, float b) { return float3(a.x - b, a.y - b, a.z - b); }
inline float3 operator-(float b, const float3 &a) { return float3(b - a.x, b - a.y, b - a.z); }
inline void operator-=(float3 &a, const float3 &b) { a.x -= b.x; a.y -= b.y; a.z -= b.z; }
inline void operator-=(float3 &a, float b) { a.x -= b; a.y -= b; a.z -= b; }
inline float3 operator*(const float3 &a, const float3 &b) { return float3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline float3 operator*(const float3 &a, float b) { return float3(a.x * b, a.y * b, a.z * b); }
inline float3 operator*(float b, const float3 &a) { return float3(b * a.x, b * a.y, b * a.z); }
inline void operator*=(float3 &a, const float3 &b) { a.x *= b.x; a.y *= b.y; a.z *= b.z; }
inline void operator*=(float3 &a, float b) { a.x *= b; a.y *= b; a.z *= b; }
inline float3 operator/(const float3 &a, const float3 &b) { return float3(a.x / b.x, a.y / b.y, a.z / b.z); }
inline float3 operator/(const float3 &a, float b) { return float3(a.x / b, a.y / b, a.z / b); }
inline float3 operator/(float b, const float3 &a) { return float3(b / a.x, b / a.y, b / a.z); }
inline void operator/=(float3 &a, const float3 &b) { a.x /= b.x; a.y /= b.y; a.z /= b.z; }
inline void operator/=(float3 &a, float b) { a.x /= b; a.y /= b; a.z /= b; }
inline float dot(const float3 &a, const float3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float3 cross(const float3 &a, const float3 &b) {
    return float3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline float sqrLength(const float3 &v) { return dot(v, v); }
inline float length(const float3 &v) { return sqrtf(dot(v, v)); }
inline float rsqrtf(float x) { return 1.0f / sqrtf(x); }
inline float3 normalize(const float3 &v) { float invLen = rsqrtf(dot(v, v)); return v * invLen; }
inline float3 reflect(const float3 &i, const float3 &n) { return i - 2.0f * n * dot(n, i); }
// the reference's select-based min / max (template/precomp.h:471-472), not C's fminf
inline float3 fminf(const float3 &a, const float3 &b) {
    return float3(a.x < b.x ? a.x : b.x, a.y < b.y ? a.y : b.y, a.z < b.z ? a.z : b.z);
}
inline float3 fmaxf(const float3 &a, const float3 &b) {
    return float3(a.x > b.x ? a.x : b.x, a.y > b.y ? a.y : b.y, a.z > b.z ? a.z : b.z);
}
inline float3 lerp(const float3 &a, const float3 &b, float t) { return a + t * (b - a); }
inline float3 clamp(const float3 &v, float a, float b) {
    auto c = [&](float f) { float m = f < b ? f : b; return a > m ? a : m; };   // fmaxf(a, fminf(f, b))
    return float3(c(v.x), c(v.y), c(v.z));
}

// ---- Surface (template/precomp.h:110-135): 0x00RRGGBB pixels
class Surface {
  public:
    Surface() = default;
    Surface(int w, int h, uint *buffer) : pixels(buffer), width(w), height(h) {}
    Surface(int w, int h) : width(w), height(h), ownBuffer(true) {
        pixels = static_cast<uint *>(std::calloc((size_t)w * h, sizeof(uint)));
        if (!pixels) throw RtError(RT_ERR_INVALID, "Surface: out of host memory");
    }
    explicit Surface(const char *file) { LoadImage(file); }   // template/template.cpp:1571-1577
    Surface(const Surface &) = delete;
    Surface &operator=(const Surface &) = delete;
    ~Surface() {
        if (ownBuffer) std::free(pixels);
    }
    void LoadImage(const char *file) {   // template/template.cpp:1579-1601 (PNG via rt_image_load)
        uint32_t *px = nullptr, w = 0, h = 0;
        rt_check(rt_image_load(file, &px, &w, &h));
        if (ownBuffer) std::free(pixels);
        pixels = px;
        width = (int)w;
        height = (int)h;
        ownBuffer = true;
    }
    void Clear(uint c) {
        for (size_t i = 0; i < (size_t)width * height; ++i) pixels[i] = c;
    }
    uint *pixels = nullptr;
    int width = 0, height = 0;
    bool ownBuffer = false;
};

// ---- application base class (template/precomp.h:1640-1654)
class TheApp {
  public:
    virtual ~TheApp() = default;
    virtual void Init() = 0;
    virtual void Tick(float deltaTime) = 0;
    virtual void Shutdown() = 0;
    virtual void MouseUp(int button) = 0;
    virtual void MouseDown(int button) = 0;
    virtual void MouseMove(int x, int y) = 0;
    virtual void MouseWheel(float y) = 0;
    virtual void KeyUp(int key) = 0;
    virtual void KeyDown(int key) = 0;
    Surface *screen = 0;
    const Surface *skydome = 0;
};

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
    // Scene() (template/scene.h:40-128): the reference's default scene, built on the device at
    // first use -- after SetSky, which Renderer::Init calls with the host's skydome
    Scene() {
        const char *dir = std::getenv("RT_MESH_DIR");
        recipe_ = "default";
        mesh_dir_ = dir ? dir : "assets";
    }
    explicit Scene(const char *recipe, const char *mesh_dir, int device = 0) : device_(device) {
        rt_check(rt_scene_create_recipe(recipe, mesh_dir, device, &h_));
    }
    explicit Scene(const rt_scene_desc &desc) { rt_check(rt_scene_create(&desc, &h_)); }
    Scene(const Scene &) = delete;
    Scene &operator=(const Scene &) = delete;
    ~Scene() { rt_scene_destroy(h_); }

    // the sky of a scene not yet on the device (power-of-two sides, renderer.h:15-22)
    void SetSky(const Surface *sky) {
        if (h_) throw RtError(RT_ERR_INVALID, "Scene::SetSky after the scene was created");
        sky_ = sky;
    }

    void IntersectBVH(Ray &ray) { std::vector<Ray *> one{&ray}; IntersectBVH(one); }
    bool IsOccluded(Ray &ray) { std::vector<Ray *> one{&ray}; return IsOccluded(one)[0]; }

    void IntersectBVH(std::vector<Ray *> &rays) {
        std::vector<rt_ray> in = pack(rays);
        std::vector<rt_hit> out(in.size());
        rt_check(rt_intersect_host(handle(), in.data(), out.data(), (uint32_t)in.size()));
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
        rt_check(rt_intersect_packets_host(handle(), in.data(), out.data(), (uint32_t)in.size()));
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
        rt_check(rt_occluded_host(handle(), in.data(), out.data(), (uint32_t)in.size()));
        return std::vector<bool>(out.begin(), out.end());
    }
    float3 GetLightColor() const { return float3(24, 24, 22); }          // template/scene.h:237-239
    float3 GetLightDir() const { return float3(0.0f, -1.0f, 0.0f); }     // template/scene.h:240-242
    rt_scene_info Info() { rt_scene_info i{}; rt_check(rt_scene_get_info(handle(), &i)); return i; }
    rt_scene *handle() {
        if (!h_) create();
        return h_;
    }

  private:
    rt_scene *h_ = nullptr;
    int device_ = 0;
    std::string recipe_, mesh_dir_;
    const Surface *sky_ = nullptr;
    void create() {   // a recipe description + the sky, on the device
        uint32_t np = 0, nm = 0;
        rt_check(rt_recipe_describe(recipe_.c_str(), mesh_dir_.c_str(), nullptr, &np, nullptr, &nm));
        std::vector<rt_prim> prims(np);
        std::vector<rt_material> mats(nm);
        rt_check(rt_recipe_describe(recipe_.c_str(), mesh_dir_.c_str(), prims.data(), &np, mats.data(), &nm));
        rt_scene_desc d{};
        d.prims = prims.data();
        d.num_prims = np;
        d.materials = mats.data();
        d.num_materials = nm;
        if (sky_ && sky_->pixels) {
            d.sky_pixels = sky_->pixels;
            d.sky_width = (uint32_t)sky_->width;
            d.sky_height = (uint32_t)sky_->height;
        }
        d.device = device_;
        rt_check(rt_scene_create(&d, &h_));
    }
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
    Camera(uint32_t width = SCRWIDTH, uint32_t height = SCRHEIGHT) { rt_check(rt_camera_default(width, height, &cam)); }
    rt_camera cam{};
};

class Renderer : public TheApp {   // renderer.h:5-160
  public:
    // `app = new Renderer()` (template/template.cpp:136): the reference's default scene; the
    // host sets screen and skydome, then calls Init() (137-139)
    Renderer() : own_(new Scene()), scene(*own_) {}
    // a renderer of a given scene and frame size, ready at once (no Init needed)
    Renderer(Scene &scene, uint32_t width, uint32_t height) : scene(scene) { create(width, height); }
    Renderer(const Renderer &) = delete;
    Renderer &operator=(const Renderer &) = delete;
    ~Renderer() override { rt_renderer_destroy(h_); }

    // Renderer::Init (renderer.cpp:6-12): the accumulator for the screen's size (SCRWIDTH x
    // SCRHEIGHT without a screen); the skydome becomes the scene's sky
    void Init() override {
        if (h_) return;
        if (skydome) scene.SetSky(skydome);
        create(screen ? (uint32_t)screen->width : SCRWIDTH, screen ? (uint32_t)screen->height : SCRHEIGHT);
    }
    // Renderer::Tick (renderer.cpp:200-309): one frame -- Trace (depth 10, renderer.h:9) or
    // WhittedTrace (depth 20, renderer.h:13) per pixel, accumulate, RGB8 into screen->pixels
    // (or `pixels` without a screen)
    void Tick(float deltaTime) override { Tick(deltaTime, 0u, 1u); }
    // the same with an explicit Trace depth (0 = the reference's default) and samples per pixel;
    // usePackets = the PACKET_TRAVERSAL build (Ray.h:3): 8x8 packets through TracePacket
    void Tick(float /*deltaTime*/, uint32_t depth, uint32_t spp = 1) {
        if (!h_) Init();
        if (depth == 0) depth = useWhitted ? 20 : 10;
        const uint32_t mode = useWhitted ? RT_MODE_WHITTED : usePackets ? RT_MODE_PACKET : RT_MODE_PATH;
        rt_frame_params p{width_, height_, spp, depth, frame_++, mode, tracerSwap ? 1u : 0u};
        tracerSwap = false;
        uint32_t *out = pixels.data();
        if (screen && screen->pixels && (uint32_t)screen->width == width_ && (uint32_t)screen->height == height_)
            out = screen->pixels;
        rt_check(rt_render_frame_host(h_, &camera.cam, &p, out));
    }
    void Shutdown() override {}
    // input (renderer.h:100-140): the K key switches integrators (138); camera motion belongs to
    // the GLFW front-end, which is out of scope, so the other events change nothing
    void MouseUp(int) override {}
    void MouseDown(int) override {}
    void MouseMove(int, int) override {}
    void MouseWheel(float) override {}
    void KeyUp(int) override {}
    void KeyDown(int key) override {
        if (key == 75) ToggleWhitted();
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
    void ToggleWhitted() { useWhitted = !useWhitted; tracerSwap = true; }
    rt_counters Counters() { rt_counters c{}; rt_check(rt_renderer_counters(h_, &c)); return c; }
    // the float4 accumulator (renderer.h:143), read back from the device
    std::vector<float4> Accumulator() {
        std::vector<float4> a((size_t)width_ * height_);
        rt_check(rt_renderer_read_accumulator(h_, &a[0].x));
        return a;
    }

  private:
    std::unique_ptr<Scene> own_;    // Renderer(): the default scene it owns

  public:
    Scene &scene;                   // renderer.h:144
    Camera camera;                  // renderer.h:145 (re-made for the frame size by Init)

  private:
    void create(uint32_t width, uint32_t height) {
        camera = Camera(width, height);
        width_ = width;
        height_ = height;
        pixels.assign((size_t)width * height, 0u);
        rt_check(rt_renderer_create(scene.handle(), width, height, &h_));
    }
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
    uint32_t width_ = 0, height_ = 0;
    uint32_t frame_ = 0;
    rt_renderer *h_ = nullptr;

  public:
    bool useWhitted = false;        // renderer.h:158
    bool tracerSwap = false;        // renderer.h:159: the next frame restarts accumulation
    bool usePackets = false;        // PACKET_TRAVERSAL, Ray.h:3
    std::vector<uint32_t> pixels;   // 0x00RRGGBB, the frame when no screen Surface is attached
};

}  // namespace Tmpl8
