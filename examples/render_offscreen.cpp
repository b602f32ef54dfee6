// render_offscreen.cpp — the reference TestProgram's frame loop (TestProgram/Program.cpp:140-340)
// written against include/beam/Beam.h, offscreen: build a scene, trace one frame, write a PPM.
//   ./render_offscreen [out.ppm [devices]]      devices: e.g. "0,1,2,3" — the frame's screen bands
//   over several GPUs (repeats allowed), gathered on the first; the default is one device.
#include <beam/Beam.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace Beam;

int main(int argc, char** argv) {
    const char* out = argc > 1 ? argv[1] : "frame.ppm";
    if (argc > 2) {  // device list, before the first Beam object
        std::vector<int> devices;
        for (const char* p = argv[2]; *p;) {
            char* end = nullptr;
            devices.push_back((int)std::strtol(p, &end, 10));
            if (end == p) return 2;
            p = *end == ',' ? end + 1 : end;
        }
        setDevices(devices);
    }
    const u32 W = 500, H = 500;  // TestProgram's window (main2.cpp:8)
    // the quad of Program.cpp:152-178 (two triangles facing -z)
    const float vertices[] = {-1.f, -1.f, 1.56f, 0.f, 1.f, 1.56f, 1.f, -1.f, 1.56f, 2.f, 1.f, 1.56f};
    const float normals[] = {0, 0, -1, 0, 0, -1, 0, 0, -1, 0.3f, 0, -1};
    const u32 indices[] = {0, 1, 2, 1, 2, 3};
    auto scene = IScene::create();
    auto mesh = IMesh::create();
    if (!scene || !mesh) {
        std::fprintf(stderr, "no device: %s\n", lastError().c_str());
        return 1;
    }
    u32 err = mesh->setIndices(indices, 6);
    err |= mesh->setVertexData(vertices, 4, 3, VERTEX_DATA_POSITION);
    err |= mesh->setVertexData(normals, 4, 3, VERTEX_DATA_NORMAL);
    scene->addMesh(mesh);
    scene->updateGPUScene();
    auto camera = ICamera::create();
    err |= camera->setInitialRays(W, H, -1, 1, -1, 1, 1);  // Program.cpp:189
    auto rt = IRenderTarget::createOffscreen(W, H);
    err |= rt->lock();
    const float eye[3] = {0.f, 0.f, -2.1f};                   // Program.cpp:106
    const float orient[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    err |= camera->traceScene(eye, orient, scene);
    std::vector<u32> px(W * H);
    err |= rt->read(px.data());
    err |= rt->unlock();
    if (err) {
        std::fprintf(stderr, "error %u: %s\n", err, lastError().c_str());
        return 1;
    }
    FILE* f = std::fopen(out, "wb");
    std::fprintf(f, "P6 %u %u 255\n", W, H);
    u32 hits = 0;
    for (u32 v : px) {
        const unsigned char rgb[3] = {(unsigned char)(v >> 16), (unsigned char)(v >> 8), (unsigned char)v};
        std::fwrite(rgb, 1, 3, f);
        hits += v != BM_MISS_PACKED;
    }
    std::fclose(f);
    std::printf("%s: %u of %u pixels hit on %u device(s)\n", out, hits, W * H, numDevices());
    return 0;
}
