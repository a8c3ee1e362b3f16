// A C++ caller of the batched tracking front end and of local BA through the
// C-ABI (include/gfslam/abi.h) and the drop-in Optimizer
// (include/gfslam/orbslam.h) only — no Python, no torch: what a
// reference-side integration (Tracking / LocalMapping threads) links against.
// Inputs written by tests/test_dropin_gpu.py:
//   <dir>/params.txt   w h fx fy cx cy nfeatures B M budget F
//   <dir>/frames.u8    F x B x h x w (frame 0 bootstraps)
//   <dir>/maps.bin     B x M gf_map_point (32 B); maps_desc.bin B x M x 32 B
//   <dir>/nmp.i32      B map sizes
//   <dir>/boot.f32     B x 16 Tcw, then B x 16 velocity
//   <dir>/ba_*.bin     one gf_ba_problem (kf_Tcw, kf_kind, kf_cam, pt_pos,
//                      edge_pt, edge_kf, edge_z, edge_is2) + ba_sizes.i32
// Outputs: seq_kp2mp.i32 / seq_tcw.f32 / seq_stats.i32 (one block per step),
// lba_*.bin for a free and a stopped LocalBundleAdjustment.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "gfslam/abi.h"
#include "gfslam/orbslam.h"

#define CK(expr)                                                                       \
    do {                                                                               \
        int _rc = (expr);                                                              \
        if (_rc) {                                                                     \
            std::fprintf(stderr, "%s failed (%d): %s\n", #expr, _rc, gf_last_error()); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

template <typename T>
static std::vector<T> load(const std::string& path, size_t n) {
    std::vector<T> v(n);
    std::ifstream(path, std::ios::binary).read(reinterpret_cast<char*>(v.data()), sizeof(T) * n);
    return v;
}

template <typename T>
static void append(const std::string& path, const T* p, size_t n) {
    std::ofstream f(path, std::ios::binary | std::ios::app);
    f.write(reinterpret_cast<const char*>(p), sizeof(T) * n);
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const std::string dir = argv[1];
    gf_frontend_params P{};
    int F = 0;
    {
        std::ifstream p(dir + "/params.txt");
        p >> P.width >> P.height >> P.fx >> P.fy >> P.cx >> P.cy >> P.nfeatures >> P.batch >> P.map_cap >>
            P.gf_budget >> F;
    }
    P.scale_factor = 1.2f;
    P.nlevels = 8;
    P.fast_th = 20;
    P.gf = 1;
    P.dt = 0.05;
    const int B = P.batch, M = P.map_cap;
    const size_t fb = (size_t)P.width * P.height;
    auto frames = load<uint8_t>(dir + "/frames.u8", (size_t)F * B * fb);
    auto maps = load<gf_map_point>(dir + "/maps.bin", (size_t)B * M);
    auto descs = load<uint8_t>(dir + "/maps_desc.bin", (size_t)B * M * 32);
    auto nmp = load<int32_t>(dir + "/nmp.i32", B);
    auto boot = load<float>(dir + "/boot.f32", (size_t)B * 32);

    gf_ctx* ctx = nullptr;
    CK(gf_ctx_create(0, &ctx));
    gf_frontend* fe = nullptr;
    CK(gf_frontend_create(ctx, &P, &fe));
    int cap = 0;
    CK(gf_frontend_capacity(fe, &cap));
    for (int b = 0; b < B; b++) {
        CK(gf_frontend_set_map(fe, b, &maps[(size_t)b * M], &descs[(size_t)b * M * 32], nmp[b]));
        CK(gf_frontend_set_rng(fe, b, 1 + b));
    }
    // Tracking: the first frame initialises, every later one is GrabImage (WORKING)
    CK(gf_frontend_bootstrap_host(fe, frames.data(), boot.data(), boot.data() + 16 * B, 0.0));
    std::vector<int32_t> kp2mp((size_t)B * cap), stats((size_t)GF_FE_NSTAT * B);
    std::vector<float> Tcw((size_t)B * 16);
    for (const char* f : {"/seq_kp2mp.i32", "/seq_tcw.f32", "/seq_stats.i32"}) std::remove((dir + f).c_str());
    for (int k = 1; k < F; k++) {
        CK(gf_frontend_step_host(fe, frames.data() + (size_t)k * B * fb));
        CK(gf_frontend_read(fe, GF_FE_KP2MP, kp2mp.data(), kp2mp.size() * 4));
        CK(gf_frontend_read(fe, GF_FE_TCW, Tcw.data(), Tcw.size() * 4));
        CK(gf_frontend_read(fe, GF_FE_STATS, stats.data(), stats.size() * 4));
        append(dir + "/seq_kp2mp.i32", kp2mp.data(), kp2mp.size());
        append(dir + "/seq_tcw.f32", Tcw.data(), Tcw.size());
        append(dir + "/seq_stats.i32", stats.data(), stats.size());
    }
    CK(gf_frontend_destroy(fe));

    // LocalMapping: LocalBundleAdjustment(pKF, &mbAbortBA) through the drop-in Optimizer
    auto sz = load<int32_t>(dir + "/ba_sizes.i32", 3);
    const int nkf = sz[0], npts = sz[1], ne = sz[2];
    ORB_SLAM::Optimizer::LocalBAWindow w;
    w.kf_Tcw = load<float>(dir + "/ba_kf_Tcw.bin", (size_t)nkf * 16);
    w.kf_kind = load<uint8_t>(dir + "/ba_kf_kind.bin", nkf);
    w.kf_cam = load<float>(dir + "/ba_kf_cam.bin", (size_t)nkf * 4);
    w.pt_pos = load<float>(dir + "/ba_pt_pos.bin", (size_t)npts * 3);
    w.edge_pt = load<int32_t>(dir + "/ba_edge_pt.bin", ne);
    w.edge_kf = load<int32_t>(dir + "/ba_edge_kf.bin", ne);
    w.edge_z = load<float>(dir + "/ba_edge_z.bin", (size_t)ne * 2);
    w.edge_inv_sigma2 = load<float>(dir + "/ba_edge_is2.bin", ne);
    ORB_SLAM::Optimizer::LocalBAWindow stopped = w;
    try {
        bool abort_ba = false;
        ORB_SLAM::Optimizer::LocalBundleAdjustment(&w, &abort_ba);
        bool abort_now = true;  // mbAbortBA raised before the call
        ORB_SLAM::Optimizer::LocalBundleAdjustment(&stopped, &abort_now);
    } catch (const ORB_SLAM::GpuError& e) {
        std::fprintf(stderr, "GpuError %d: %s\n", e.code, e.what());
        return 1;
    }
    for (auto* r : {&w, &stopped}) {
        const std::string s = r == &w ? "free" : "stop";
        for (const char* f : {"_T.f32", "_X.f32", "_out.u8", "_it.i32"}) std::remove((dir + "/lba_" + s + f).c_str());
        append(dir + "/lba_" + s + "_T.f32", r->kf_Tcw.data(), r->kf_Tcw.size());
        append(dir + "/lba_" + s + "_X.f32", r->pt_pos.data(), r->pt_pos.size());
        append(dir + "/lba_" + s + "_out.u8", r->edge_outlier.data(), r->edge_outlier.size());
        append(dir + "/lba_" + s + "_it.i32", r->iterations, 2);
    }
    CK(gf_ctx_destroy(ctx));
    std::printf("ok %d steps, local BA iterations %d %d (stopped %d %d)\n", F - 1, w.iterations[0], w.iterations[1],
                stopped.iterations[0], stopped.iterations[1]);
    return 0;
}
