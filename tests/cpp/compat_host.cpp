// A host written against the reference's class surface (renderer.h, template/scene.h,
// Ray.h), switched to librtamd.so through include/rt_compat.hpp.  Exit codes: 0 = all
// checks passed, 3 = no GPU (RT_ERR_NO_DEVICE, the expected outcome on a CPU-only host),
// 1 = a check failed.
#include <cmath>
#include <cstdio>

#include "rt_compat.hpp"

using namespace Tmpl8;

int main(int argc, char **argv) {
    const char *data = argc > 1 ? argv[1] : "advancedgraphicsraytracer_amd/data";
    try {
        Scene scene("teapotF", data);
        // one ray straight down the view axis hits the teapot (template/scene.h:285)
        Ray r(float3{0, 0, -1}, float3{0, 0, 1});
        scene.IntersectBVH(r);
        if (r.objIdx < 1 || !(r.t > 1 && r.t < 4)) { std::printf("IntersectBVH: obj %d t %g\n", r.objIdx, r.t); return 1; }
        Ray down(float3{0, 0.5f, 2}, float3{0, -1, 0}, 0.3f);   // inside the teapot's bounds, short
        (void)scene.IsOccluded(down);
        // a packet of 64 parallel rays, 8x8 grid (template/scene.h:322)
        RayPacket p;
        for (int i = 0; i < PACKET_SIZE; ++i) {
            p.O[i] = float3{-0.35f + 0.1f * (i & 7), -0.35f + 0.1f * (i >> 3), -1};
            p.D[i] = float3{0, 0, 1};
        }
        scene.IntersectBVHPacket(p);
        std::vector<Ray> singles(PACKET_SIZE);
        std::vector<Ray *> ptrs;
        for (int i = 0; i < PACKET_SIZE; ++i) singles[i] = Ray(p.O[i], p.D[i]), ptrs.push_back(&singles[i]);
        scene.IntersectBVH(ptrs);
        for (int i = 0; i < PACKET_SIZE; ++i)
            if (singles[i].objIdx != p.objIdx[i] || singles[i].t != p.t[i]) { std::printf("packet lane %d differs\n", i); return 1; }
        // Renderer::Tick in the three integrators
        Renderer renderer(scene, 128, 72);
        renderer.Tick(0.0f);                        // path tracer, depth 10
        uint64_t sum_pt = 0;
        for (uint32_t px : renderer.pixels) sum_pt += px & 0xff;
        renderer.ToggleWhitted();                   // the K key
        renderer.Tick(0.0f);                        // Whitted, depth 20
        renderer.useWhitted = false;
        renderer.usePackets = true;
        renderer.Tick(0.0f);
        rt_counters c = renderer.Counters();
        if (c.frames != 3 || c.primary != 3ull * 128 * 72 || sum_pt == 0) {
            std::printf("counters: frames %llu primary %llu\n", (unsigned long long)c.frames, (unsigned long long)c.primary);
            return 1;
        }
        std::printf("compat host ok: obj %d t %.4f shadow %llu bounce %llu\n", r.objIdx, r.t,
                    (unsigned long long)c.shadow, (unsigned long long)c.bounce);
        return 0;
    } catch (const RtError &e) {
        std::printf("RtError %d: %s\n", e.code, e.what());
        return e.code == RT_ERR_NO_DEVICE ? 3 : 1;
    }
}
