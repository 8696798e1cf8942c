// A host shaped like the reference's own main (template/template.cpp:133-139, 269-287) and
// its vector math, with the reference's `#include "precomp.h"` swapped for rt_compat.hpp and
// nothing else: screen / skydome Surfaces, `app = new Renderer()`, Init, a Tick loop, the K
// key, Shutdown.  Renderer() builds the reference's default scene (template/scene.h:40-128)
// from $RT_MESH_DIR.  Exit 0 = the frames came back and the checks passed, 3 = no GPU
// (RT_ERR_NO_DEVICE: the expected outcome on a CPU-only host), 1 = a check failed.
#include <cstdio>

#include "rt_compat.hpp"   // was: #include "precomp.h"

using namespace Tmpl8;

static TheApp *app = 0;

int main(int argc, char **argv) {
    try {
        // float3 arithmetic as the reference's host code writes it (template/precomp.h:569-855)
        float3 a(1, 2, 3), b = float3(0.5f);
        a += b * 2.0f;
        a -= float3(1, 1, 1);
        float3 n = normalize(cross(a, float3(0, 1, 0)));
        float3 r = reflect(float3(1, -1, 0), float3(0, 1, 0));
        if (a.x != 1 || a.y != 2 || a.z != 3 || r.y != 1 || std::fabs(length(n) - 1.0f) > 1e-6f || dot(n, a) > 1e-5f ||
            fminf(a, float3(2)).z != 2 || fmaxf(a, float3(2)).x != 2 || (a / 2.0f).y != 1 || (-a)[0] != -1) {
            std::printf("float3 operators\n");
            return 1;
        }
        // initialize application (template/template.cpp:133-139)
        Surface *screen = new Surface(SCRWIDTH / 4, SCRHEIGHT / 4);
        Surface *skydome = argc > 1 ? new Surface(argv[1]) : new Surface(1024, 512);   // power of two (renderer.h:18)
        if (argc <= 1) skydome->Clear(0x406080);
        app = new Renderer();
        app->screen = screen;
        app->skydome = skydome;
        app->Init();
        // main loop (template/template.cpp:269-286)
        float deltaTime = 0;
        for (int frameNr = 0; frameNr < 3; ++frameNr) {
            app->Tick(deltaTime);
            deltaTime = 16.0f;
        }
        uint64_t sum = 0;
        for (int i = 0; i < screen->width * screen->height; ++i) sum += screen->pixels[i] & 0xffffff;
        app->KeyDown(75);   // K: Whitted (renderer.h:138)
        app->Tick(deltaTime);
        Renderer *rend = static_cast<Renderer *>(app);
        rt_counters c = rend->Counters();
        rt_scene_info info = rend->scene.Info();
        // the default scene: light + glider (21,364 triangles) + mig29 (6,546)
        if (sum == 0 || c.frames != 4 || info.num_prims != 1 + 21364 + 6546 || !rend->useWhitted) {
            std::printf("frames %llu prims %u sum %llu\n", (unsigned long long)c.frames, info.num_prims, (unsigned long long)sum);
            return 1;
        }
        app->Shutdown();   // close down (template/template.cpp:287)
        delete app;
        delete skydome;
        delete screen;
        std::printf("reference-shaped host ok: %u prims, %llu primary rays\n", info.num_prims, (unsigned long long)c.primary);
        return 0;
    } catch (const RtError &e) {
        std::printf("RtError %d: %s\n", e.code, e.what());
        return e.code == RT_ERR_NO_DEVICE ? 3 : 1;
    }
}
