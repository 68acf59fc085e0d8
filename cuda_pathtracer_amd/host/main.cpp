// pathtracer_amd — headless restatement of the reference's main loop (path_tracer/src/main.cpp):
// load the scene, InitDataContainer, then runCuda's sequence (main.cpp:114-168) without the GL
// window — pathtraceInit, `iterations` calls of pathtrace(), saveImage() (main.cpp:88-112) and
// pathtraceFree().  The camera is the first-frame orbit recompute (done by pt_scene_finalize).
//
//   pathtracer_amd SCENEFILE.json [--iterations N] [--out DIR] [--sort] [--no-png] [--hdr]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <sstream>
#include <string>

#include "pathtrace.h"

namespace {

std::string currentTimeString() {   // preview.cpp:21-28
    time_t now;
    time(&now);
    char buf[sizeof "0000-00-00_00-00-00z"];
    strftime(buf, sizeof buf, "%Y-%m-%d_%H-%M-%Sz", gmtime(&now));
    return std::string(buf);
}

// saveImage (main.cpp:88-112): divide by the sample count, mirror x, clamp, x255, PNG.
std::string saveImage(const Scene& scene, const std::string& dir, const std::string& start, int iteration,
                      bool hdr = false) {
    const float samples = (float)iteration;
    std::ostringstream ss;
    ss << scene.state.imageName << "." << start << "." << samples << "samp";
    std::string filename = ss.str();
    if (!dir.empty()) filename = dir + "/" + filename;
    filename += hdr ? ".hdr" : ".png";   // Image::savePNG / saveHDR append the extension (image.cpp:22-49)
    const int W = scene.state.camera.res[0], H = scene.state.camera.res[1];
    const float* rgb = reinterpret_cast<const float*>(scene.state.image.data());
    if (hdr ? pt_save_hdr(filename.c_str(), rgb, W, H, samples) : pt_save_png(filename.c_str(), rgb, W, H, samples)) {
        std::fprintf(stderr, "saveImage: %s\n", pt_last_error());
        std::exit(EXIT_FAILURE);
    }
    return filename;
}

}  // namespace

int main(int argc, char** argv) {
    const std::string startTimeString = currentTimeString();
    if (argc < 2) {
        std::printf("Usage: %s SCENEFILE.json [--iterations N] [--out DIR] [--sort] [--no-png] [--hdr]\n", argv[0]);
        return 1;
    }
    const char* sceneFile = argv[1];
    int iterations = -1;
    std::string out_dir;
    bool sort = false, png = true, hdr = false;
    for (int i = 2; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--iterations") && i + 1 < argc) iterations = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--out") && i + 1 < argc) out_dir = argv[++i];
        else if (!std::strcmp(argv[i], "--sort")) sort = true;
        else if (!std::strcmp(argv[i], "--no-png")) png = false;
        else if (!std::strcmp(argv[i], "--hdr")) hdr = true;   // also write the saveHDR .hdr file
        else {
            std::fprintf(stderr, "unknown argument %s\n", argv[i]);
            return 1;
        }
    }

    Scene* scene = new Scene(sceneFile);
    GuiDataContainer* guiData = new GuiDataContainer();
    guiData->sortbyMaterial = sort;
    InitDataContainer(guiData);
    const int total = iterations > 0 ? iterations : (int)scene->state.iterations;

    pathtraceInit(scene);
    const auto t0 = std::chrono::steady_clock::now();
    int iteration = 0;
    while (iteration < total) {
        ++iteration;
        pathtrace(nullptr, 0, iteration);
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    pt_stats_t st{};
    (void)st;
    std::printf("rendered %d iteration(s) of %s (%dx%d, depth %d) in %.3f s\n", iteration, sceneFile,
                scene->state.camera.res[0], scene->state.camera.res[1], scene->state.traceDepth, secs);
    if (png) std::printf("wrote %s\n", saveImage(*scene, out_dir, startTimeString, iteration).c_str());
    if (hdr) std::printf("wrote %s\n", saveImage(*scene, out_dir, startTimeString, iteration, true).c_str());
    pathtraceFree();
    delete guiData;
    delete scene;
    return 0;
}
