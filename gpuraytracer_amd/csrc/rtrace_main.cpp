// rtrace_main.cpp — C++ host of record (Swift is unavailable on this image).
//
// Mirrors the reference's live entry point and host class:
//   RTrace/main.swift:13-30      output path = argv[1] or "output.png"; Renderer(); draw()
//   RTrace/renderer.swift        class Renderer { init(); draw() }
//   RTrace/image.swift:15-100    saveTextureToImage -> tonemapped RGBA8 PNG
// on top of the C-ABI (include/rtpt.h).  Extra flags replace the reference's
// hard-coded constants (raytrace.metal:24-25, scene.swift:18, renderer.swift:100):
//   rtrace [out.png] [--res WxH] [--spp N] [--batch N] [--bounces B]
//          [--scene cornell|spheres:N] [--seed KEY] [--device D] [--pfm out.pfm]
//   rtrace --mis [out.png] [--res WxH] [--camera-rays N] [--mis-samples N]
//          the SwiftPM build (Sources/gpuRaytracer/main.swift:96-108): scene with the
//          1.5 x 1.5 light, kernel drawTriangle (6 camera rays x 300 MIS samples),
//          its own tonemapped RGBA8 written as the PNG
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "../../include/rtpt.h"

namespace {

// Minimal PNG writer (stored deflate blocks): no zlib on the image.
uint32_t crc32(const uint8_t* d, size_t n, uint32_t c = 0xFFFFFFFFu) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t r = i;
            for (int k = 0; k < 8; ++k) r = (r & 1) ? 0xEDB88320u ^ (r >> 1) : r >> 1;
            table[i] = r;
        }
        init = true;
    }
    for (size_t i = 0; i < n; ++i) c = table[(c ^ d[i]) & 0xFF] ^ (c >> 8);
    return c;
}

void put32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24)); v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8)); v.push_back((uint8_t)x);
}

void chunk(FILE* f, const char* type, const std::vector<uint8_t>& data) {
    std::vector<uint8_t> buf;
    put32(buf, (uint32_t)data.size());
    buf.insert(buf.end(), type, type + 4);
    buf.insert(buf.end(), data.begin(), data.end());
    const uint32_t c = crc32(buf.data() + 4, buf.size() - 4) ^ 0xFFFFFFFFu;
    put32(buf, c);
    fwrite(buf.data(), 1, buf.size(), f);
}

bool write_png(const char* path, const uint8_t* rgba, int w, int h) {
    FILE* f = fopen(path, "wb");
    if (!f) return false;
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    fwrite(sig, 1, 8, f);
    std::vector<uint8_t> ihdr;
    put32(ihdr, (uint32_t)w);
    put32(ihdr, (uint32_t)h);
    ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // 8-bit RGBA
    chunk(f, "IHDR", ihdr);
    std::vector<uint8_t> raw;
    raw.reserve((size_t)h * (4 * (size_t)w + 1));
    for (int y = 0; y < h; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), rgba + (size_t)y * 4 * w, rgba + (size_t)(y + 1) * 4 * w);
    }
    std::vector<uint8_t> z = {0x78, 0x01};
    uint32_t a = 1, b = 0;
    for (uint8_t v : raw) { a = (a + v) % 65521u; b = (b + a) % 65521u; }
    for (size_t off = 0; off < raw.size() || off == 0; off += 65535) {
        const size_t n = raw.size() - off < 65535 ? raw.size() - off : 65535;
        const bool last = off + n >= raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back((uint8_t)n); z.push_back((uint8_t)(n >> 8));
        z.push_back((uint8_t)~n); z.push_back((uint8_t)(~n >> 8));
        z.insert(z.end(), raw.begin() + off, raw.begin() + off + n);
        if (last) break;
    }
    put32(z, (b << 16) | a);
    chunk(f, "IDAT", z);
    chunk(f, "IEND", {});
    return fclose(f) == 0;
}

bool write_pfm(const char* path, const float* rgba, int w, int h) {
    FILE* f = fopen(path, "wb");
    if (!f) return false;
    fprintf(f, "PF\n%d %d\n-1.0\n", w, h);
    std::vector<float> row(3 * (size_t)w);
    for (int y = h - 1; y >= 0; --y) {  // PFM stores bottom row first
        for (int x = 0; x < w; ++x)
            for (int c = 0; c < 3; ++c) row[3 * x + c] = rgba[4 * ((size_t)y * w + x) + c];
        fwrite(row.data(), sizeof(float), row.size(), f);
    }
    return fclose(f) == 0;
}

// class Renderer (RTrace/renderer.swift:9-187)
class Renderer {
   public:
    struct Options {
        int width = 800, height = 600;   // scene.swift:18
        uint32_t spp = 400, bounces = 3;  // raytrace.metal:24-25
        uint32_t batch = 0;               // spp per launch (0 = all at once)
        uint32_t spheres = 0;             // 0 = Cornell box
        uint64_t seed_key = 0x5EED00000000ull;
        int device = 0;
        bool mis = false;                 // SwiftPM drawTriangle instead of pathTrace
        uint32_t camera_rays = 6, mis_samples = 300;  // shaders.metal:644-649
    };

    explicit Renderer(const Options& o) : opt_(o) {  // Renderer.init() :29-115
        std::vector<MaterialGPU> mats;
        std::vector<rt_float3> verts;
        uint32_t n_tri = 0;
        if (o.spheres) {
            mats.resize(RT_SPHERE_SCENE_TRIANGLES);
            verts.resize(3 * RT_SPHERE_SCENE_TRIANGLES);
            spheres_.resize(o.spheres);
            rt_scene_random_spheres(o.width, o.height, o.spheres, 42, &camera_, mats.data(),
                                    verts.data(), &light_, &n_tri, spheres_.data());
        } else if (o.mis) {
            mats.resize(RT_CORNELL_TRIANGLES);
            verts.resize(3 * RT_CORNELL_TRIANGLES);
            rt_scene_cornell_box_mis(o.width, o.height, &camera_, mats.data(), verts.data(),
                                     &light_, &n_tri);
        } else {
            mats.resize(RT_CORNELL_TRIANGLES);
            verts.resize(3 * RT_CORNELL_TRIANGLES);
            rt_scene_cornell_box(o.width, o.height, &camera_, mats.data(), verts.data(), &light_,
                                 &n_tri);
        }
        rt_scene_desc d;
        memset(&d, 0, sizeof(d));
        d.camera = &camera_;
        d.materials = mats.data();
        d.square_lights = &light_;
        d.n_square_lights = 1;
        d.vertices = verts.data();
        d.n_triangles = n_tri;
        d.spheres = spheres_.empty() ? nullptr : spheres_.data();
        d.n_spheres = (uint32_t)spheres_.size();
        d.device = o.device;
        check(rt_create(&d, &ctx_), nullptr);
        check(rt_fill_seeds(ctx_, o.seed_key), ctx_);  // renderer.swift:96-110
    }
    ~Renderer() { rt_destroy(ctx_); }

    // Renderer.draw() (:117-146) followed by saveTextureToImage's tonemap
    // (image.swift:35-65): with rgba8 the kernel stores the 8-bit image itself
    // (RT_OUT_RGBA8, the epilogue fused into its store); otherwise the fp32
    // frame.  Returns kernel seconds.
    double draw(std::vector<float>* image, std::vector<uint8_t>* rgba8 = nullptr) {
        const size_t px = (size_t)opt_.width * opt_.height;
        if (rgba8) rgba8->assign(4 * px, 0);
        else image->assign(4 * px, 0.0f);
        void* out = rgba8 ? (void*)rgba8->data() : (void*)image->data();
        const uint32_t batch = opt_.batch ? opt_.batch : opt_.spp;
        double kernel_s = 0.0;
        for (uint32_t base = 0; base < opt_.spp; base += batch) {
            rt_render_params p;
            memset(&p, 0, sizeof(p));
            p.spp = (opt_.spp - base < batch) ? opt_.spp - base : batch;
            p.bounces = opt_.bounces;
            p.sample_base = base;
            p.accumulate = base > 0;
            const bool last = base + p.spp >= opt_.spp;
            p.flags = (last ? (rgba8 ? RT_OUT_RGBA8 : 0u) : RT_OUT_NONE) | (opt_.batch ? RT_KEEP_SUM : 0u);
            check(rt_render(ctx_, &p, last ? out : nullptr), ctx_);
            float ms = 0;
            check(rt_last_kernel_ms(ctx_, &ms), ctx_);
            kernel_s += ms * 1e-3;
        }
        return kernel_s;
    }

    // drawTriangle(device:...) (Sources/gpuRaytracer/computeShader.swift:99-189):
    // radiance sums and the kernel's own RGBA8; returns kernel seconds
    double draw_mis(std::vector<float>* sums, std::vector<uint8_t>* rgba8) {
        sums->assign((size_t)opt_.width * opt_.height * 4, 0.0f);
        rgba8->assign((size_t)opt_.width * opt_.height * 4, 0);
        rt_mis_params p;
        memset(&p, 0, sizeof(p));
        p.camera_rays = opt_.camera_rays;
        p.mis_samples = opt_.mis_samples;
        check(rt_render_mis(ctx_, &p, sums->data(), rgba8->data()), ctx_);
        float ms = 0;
        check(rt_last_kernel_ms(ctx_, &ms), ctx_);
        return ms * 1e-3;
    }

   private:
    static void check(int s, rt_ctx* c) {
        if (s != RT_OK) {
            fprintf(stderr, "rtrace: %s: %s\n", rt_status_string(s), rt_last_error(c));
            exit(1);
        }
    }
    Options opt_;
    CameraGPU camera_;
    SquareLightGPU light_;
    std::vector<SphereGPU> spheres_;
    rt_ctx* ctx_ = nullptr;
};

}  // namespace

int main(int argc, char** argv) {
    Renderer::Options o;
    std::string out = "output.png", pfm;  // main.swift:13-26
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) { fprintf(stderr, "missing value for %s\n", a.c_str()); exit(2); }
            return argv[++i];
        };
        if (a == "--res") {
            if (sscanf(next(), "%dx%d", &o.width, &o.height) != 2) { fprintf(stderr, "bad --res\n"); return 2; }
        } else if (a == "--spp") o.spp = (uint32_t)strtoul(next(), nullptr, 10);
        else if (a == "--batch") o.batch = (uint32_t)strtoul(next(), nullptr, 10);
        else if (a == "--bounces") o.bounces = (uint32_t)strtoul(next(), nullptr, 10);
        else if (a == "--seed") o.seed_key = strtoull(next(), nullptr, 0);
        else if (a == "--device") o.device = atoi(next());
        else if (a == "--pfm") pfm = next();
        else if (a == "--mis") o.mis = true;
        else if (a == "--camera-rays") o.camera_rays = (uint32_t)strtoul(next(), nullptr, 10);
        else if (a == "--mis-samples") o.mis_samples = (uint32_t)strtoul(next(), nullptr, 10);
        else if (a == "--scene") {
            const std::string s = next();
            if (s.rfind("spheres:", 0) == 0) o.spheres = (uint32_t)strtoul(s.c_str() + 8, nullptr, 10);
            else if (s != "cornell") { fprintf(stderr, "unknown scene %s\n", s.c_str()); return 2; }
        } else if (a.size() && a[0] != '-') out = a;
        else { fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
    }
    if (o.mis && o.spheres) { fprintf(stderr, "--mis renders the SwiftPM Cornell scene only\n"); return 2; }
    Renderer r(o);
    if (o.mis) {  // Sources/gpuRaytracer/main.swift:96-108
        std::vector<float> sums;
        std::vector<uint8_t> rgba8;
        const auto t0 = std::chrono::steady_clock::now();
        const double ks = r.draw_mis(&sums, &rgba8);
        const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (!write_png(out.c_str(), rgba8.data(), o.width, o.height)) {
            fprintf(stderr, "failed to write %s\n", out.c_str());
            return 1;
        }
        if (!pfm.empty() && !write_pfm(pfm.c_str(), sums.data(), o.width, o.height)) return 1;
        printf("Image saved to: %s\n", out.c_str());  // image.swift:89
        printf("Render completed in %.2f seconds\n", wall);  // main.swift:106
        printf("{\"res\": \"%dx%d\", \"camera_rays\": %u, \"mis_samples\": %u, \"kernel_s\": %.6f}\n",
               o.width, o.height, o.camera_rays, o.mis_samples, ks);
        return 0;
    }
    // The PNG is the kernel's fused RGBA8 store; with --pfm the fp32 frame is
    // kept and tonemapped on the host instead (rt_tonemap_rgba8: same bytes).
    std::vector<float> img;
    std::vector<uint8_t> rgba8;
    const auto t0 = std::chrono::steady_clock::now();
    const double ks = pfm.empty() ? r.draw(&img, &rgba8) : r.draw(&img);
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!pfm.empty()) {
        rgba8.resize((size_t)o.width * o.height * 4);
        rt_tonemap_rgba8(img.data(), (size_t)o.width * o.height, rgba8.data());
    }
    if (!write_png(out.c_str(), rgba8.data(), o.width, o.height)) {
        fprintf(stderr, "failed to write %s\n", out.c_str());
        return 1;
    }
    if (!pfm.empty() && !write_pfm(pfm.c_str(), img.data(), o.width, o.height)) return 1;
    const double samples = (double)o.width * o.height * o.spp;
    printf("Image saved successfully to %s\n", out.c_str());  // image.swift:93
    printf("{\"res\": \"%dx%d\", \"spp\": %u, \"bounces\": %u, \"kernel_s\": %.6f, \"wall_s\": %.6f, "
           "\"msamples_per_s\": %.2f}\n",
           o.width, o.height, o.spp, o.bounces, ks, wall, samples / ks / 1e6);
    return 0;
}
