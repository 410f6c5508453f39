// Microbenchmark of the discriminator Conv2d kernels (csrc/disc.hip, msstftd.py:67-104) on the
// config-3 layer shapes (B = 32): every tile / loop variant against the round-1 launch
// configuration, outputs compared element-wise, time per call from hipEvents over 10 calls.
// Build: make -C tools/mb c2_mb ; run: tools/mb/c2_mb [layer filter substring]
#include "../../encodec-pytorch_amd/csrc/disc.hip"

#include <stdio.h>
#include <string.h>
#include <vector>
#include <functional>

// the library's profiler scope is compiled out here
encx_prof_scope::encx_prof_scope(hipStream_t s, double, double, const char*, bool) : st(s), slot(-1) {}
encx_prof_scope::~encx_prof_scope() {}
void encx_prof_scope::tag(const char*, ...) {}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static float* dev_rand(size_t n, unsigned seed, float scale) {
    std::vector<float> h(n);
    unsigned s = seed * 2654435761u + 1;
    for (size_t i = 0; i < n; ++i) {
        s = s * 1664525u + 1013904223u;
        h[i] = scale * ((float)((s >> 8) & 0xFFFF) / 32768.f - 1.f);
    }
    float* d;
    CK(hipMalloc(&d, n * 4));
    CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    return d;
}
static float* dev_zero(size_t n) {
    float* d;
    CK(hipMalloc(&d, n * 4));
    CK(hipMemset(d, 0, n * 4));
    return d;
}
static double rel_err(const float* a, const float* b, size_t n) {
    std::vector<float> x(n), y(n);
    CK(hipMemcpy(x.data(), a, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(y.data(), b, n * 4, hipMemcpyDeviceToHost));
    double m = 0, d = 0;
    for (size_t i = 0; i < n; ++i) {
        m = fmax(m, fabs((double)y[i]));
        d = fmax(d, fabs((double)x[i] - (double)y[i]));
    }
    return d / (m + 1e-30);
}
static double time_ms(std::function<void()> f, int reps = 10) {
    f();
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

struct Layer {
    const char* name;
    int Ci, Co, T2, Fi, KT, KF, sf, dt;
};

int main(int argc, char** argv) {
    const char* filt = argc > 1 ? argv[1] : "";
    const int B = 32;
    // disc k: spectrogram (T2 frames, F bins) -> L0 s1 -> L1..L3 s2 (dil 1,2,4) -> L4 3x3 -> post 3x3
    const int T2s[3] = {90, 43, 184}, Fs[3] = {513, 1025, 257};
    std::vector<Layer> L;
    static char names[64][48];
    int nn = 0;
    for (int d = 0; d < 3; ++d) {
        int F = Fs[d];
        snprintf(names[nn], 48, "d%d L0 2x32 F%d", d, F);
        L.push_back({names[nn++], 2, 32, T2s[d], F, 3, 9, 1, 1});
        for (int l = 1; l <= 3; ++l) {
            snprintf(names[nn], 48, "d%d L%d 32x32 F%d", d, l, F);
            L.push_back({names[nn++], 32, 32, T2s[d], F, 3, 9, 2, 1 << (l - 1)});
            F = (F + 8 - 9) / 2 + 1;
        }
        snprintf(names[nn], 48, "d%d L4 32x32 3x3 F%d", d, F);
        L.push_back({names[nn++], 32, 32, T2s[d], F, 3, 3, 1, 1});
        snprintf(names[nn], 48, "d%d post 32x1 F%d", d, F);
        L.push_back({names[nn++], 32, 1, T2s[d], F, 3, 3, 1, 1});
    }
    hipStream_t st = 0;
    double tot_old[3] = {0, 0, 0}, tot_new[3] = {0, 0, 0};
    for (const Layer& l : L) {
        if (!strstr(l.name, filt)) continue;
        const int pt = (l.KT - 1) * l.dt / 2, pf = (l.KF - 1) / 2;
        const int Fo = (l.Fi + 2 * pf - l.KF) / l.sf + 1;
        C2Geo g{B, l.Ci, l.T2, l.Fi, l.Co, Fo, l.KT, l.KF, l.sf, l.dt, pt, pf};
        const size_t nx = (size_t)B * l.Ci * l.T2 * l.Fi, ny = (size_t)B * l.Co * l.T2 * Fo;
        const size_t nw = (size_t)l.Co * l.Ci * l.KT * l.KF;
        const double flops = 2.0 * B * l.Co * l.T2 * Fo * l.Ci * l.KT * l.KF;
        float* x = dev_rand(nx, 1, 1.f);
        float* wf = dev_rand(nw, 2, 0.05f);
        float* bias = dev_rand(l.Co, 3, 0.1f);
        float* y0 = dev_zero(ny);
        float* y1 = dev_zero(ny);
        float* dy = dev_rand(ny, 4, 1.f);
        float* yact = dev_rand(ny, 5, 1.f);
        float* dx0 = dev_zero(nx);
        float* dx1 = dev_zero(nx);
        const int J = (l.KF + l.sf - 1) / l.sf;
        float* wp = dev_zero((size_t)l.Co * l.KT * J * l.Ci * l.sf);
        hipLaunchKernelGGL(c2_wpoly_kernel, dim3((unsigned)cdiv((int64_t)l.Co * l.KT * J * l.Ci * l.sf, 256)), dim3(256), 0,
                           st, wf, wp, l.Co, l.Ci, l.KT, l.KF, l.sf, J);
        printf("== %s  T2=%d Fo=%d  %.2f GFLOP per call\n", l.name, l.T2, Fo, flops * 1e-9);
        const char* only = getenv("MB_ONLY");  // fwd | dgrad | wgrad
        // ---- forward
        if (!only || !strcmp(only, "fwd")) {
            C2Fwd a{g, x, wf, bias, y0, 1, 0, 0, 0};
            auto old = [&] { run_fwd<32, 128, 1, 4>(a, st); };
            double t0 = time_ms(old);
            printf("  fwd  old <32,128,1,4>        %8.1f us  %6.1f TF/s\n", t0 * 1e3, flops / t0 * 1e-9);
            tot_old[0] += t0;
            double best = t0;
            C2Fwd b = a;
            b.y = y1;
            auto var = [&](const char* nm, std::function<void()> f) {
                CK(hipMemset(y1, 0, ny * 4));
                double t = time_ms(f);
                double e = rel_err(y1, y0, ny);
                printf("  fwd  %-24s %8.1f us  %6.1f TF/s  err %.1e%s\n", nm, t * 1e3, flops / t * 1e-9, e,
                       e > 1e-5 ? "  MISMATCH" : "");
                if (e <= 1e-5 && t < best) best = t;
            };
            if (fwr_ok(g)) {
                for (int v : {0, 1}) {
                    char nm[32];
                    snprintf(nm, 32, "rw variant %d", v);
                    var(nm, [&] { if (run_fwd_rw(b, 256, st, v)) printf("    (n/a)\n"); });
                }
            }
            if (l.Co <= 32) {
                if (l.KF == 9) {
                    var("r<256,9,6,16>", [&] { if (run_fwdr<256, 9, 6, 16>(b, st)) printf("    (n/a)\n"); });
                    if (l.Ci == 2) {
                        var("<32,128,1,4,KF9>", [&] { run_fwd<32, 128, 1, 4, 9>(b, st); });
                        var("<32,256,1,4>", [&] { run_fwd<32, 256, 1, 4>(b, st); });
                        var("<32,256,1,4,KF9>", [&] { run_fwd<32, 256, 1, 4, 9>(b, st); });
                        var("r<256,9,4,16,2>", [&] { if (run_fwdr<256, 9, 4, 16, 2>(b, st)) printf("    (n/a)\n"); });
                        var("r<256,9,3,16,3>", [&] { if (run_fwdr<256, 9, 3, 16, 3>(b, st)) printf("    (n/a)\n"); });
                        var("r<128,9,2,16,4>", [&] { if (run_fwdr<128, 9, 2, 16, 4>(b, st)) printf("    (n/a)\n"); });
                    }

                } else {
                    var("r<256,3,8,32>", [&] { if (run_fwdr<256, 3, 8, 32>(b, st)) printf("    (n/a)\n"); });
                    var("r<256,3,6,32>", [&] { if (run_fwdr<256, 3, 6, 32>(b, st)) printf("    (n/a)\n"); });
                    var("q<256,3,8,32>", [&] { if (run_fwdq<256, 3, 8, 32>(b, st)) printf("    (n/a)\n"); });
                    var("q<256,3,12,32>", [&] { if (run_fwdq<256, 3, 12, 32>(b, st)) printf("    (n/a)\n"); });
                    var("v<256,3,16>", [&] { run_fwdv<256, 3, 16>(b, st); });
                    var("v<256,3,8>", [&] { run_fwdv<256, 3, 8>(b, st); });
                    var("v<512,3,8>", [&] { run_fwdv<512, 3, 8>(b, st); });
                    var("p<256,3,8,16>", [&] { if (run_fwdp<256, 3, 8, 16>(b, st)) printf("    (n/a)\n"); });
                }
            }
            tot_new[0] += best;
        }
        // ---- backward data
        if (!(l.sf == 1 && l.KF == 9) && !getenv("MB_SKIP_DGRAD") && (!only || !strcmp(only, "dgrad"))) {  // the narrow first layer has its own VALU kernel
            C2Dg a{g, dy, yact, wp, nullptr, dx0, 0, 0, 0, 0, 0, 0};
            const int M = l.Ci * l.sf;
            double t0;
            if (M > 32) t0 = time_ms([&] { run_dgrad<64, 128, 2, 2>(a, st); });
            else t0 = time_ms([&] { run_dgrad<32, 128, 1, 4>(a, st); });
            printf("  dgrad old                    %8.1f us  %6.1f TF/s\n", t0 * 1e3, flops / t0 * 1e-9);
            tot_old[1] += t0;
            double best = t0;
            C2Dg b = a;
            b.dx = dx1;
            auto var = [&](const char* nm, std::function<void()> f) {
                CK(hipMemset(dx1, 0, nx * 4));
                double t = time_ms(f);
                double e = rel_err(dx1, dx0, nx);
                printf("  dgrad %-23s %8.1f us  %6.1f TF/s  err %.1e%s\n", nm, t * 1e3, flops / t * 1e-9, e,
                       e > 1e-5 ? "  MISMATCH" : "");
                if (e <= 1e-5 && t < best) best = t;
            };
            if (dgr_ok(g)) {
                for (int v : {0, 1, 2, 3}) {
                    char nm[32];
                    snprintf(nm, 32, "rw variant %d", v);
                    var(nm, [&] { if (run_dgrad_rw(b, 256, st, v)) printf("    (n/a)\n"); });
                }
            }
            if (M == 64 && J == 5) {
                var("r<2,256,5,4,8,3>", [&] { if (run_dgradr<2, 256, 5, 4, 8, 3>(b, st)) printf("    (n/a)\n"); });
                var("r<2,256,5,4,8,3,SP>", [&] { if (run_dgradr<2, 256, 5, 4, 8, 3, 2>(b, st)) printf("    (n/a)\n"); });
                var("r<2,256,5,4,8,2,SP>", [&] { if (run_dgradr<2, 256, 5, 4, 8, 2, 2>(b, st)) printf("    (n/a)\n"); });
                var("r<2,256,5,4,16,2,SP>", [&] { if (run_dgradr<2, 256, 5, 4, 16, 2, 2>(b, st)) printf("    (n/a)\n"); });
                var("r<2,128,5,4,16,3>", [&] { if (run_dgradr<2, 128, 5, 4, 16, 3>(b, st)) printf("    (n/a)\n"); });
                var("r<2,128,5,4,16,3,SP>", [&] { if (run_dgradr<2, 128, 5, 4, 16, 3, 2>(b, st)) printf("    (n/a)\n"); });
                b.yact = nullptr;
                var("r<2,256,5,4,8,3> noY", [&] { if (run_dgradr<2, 256, 5, 4, 8, 3>(b, st)) printf("    (n/a)\n"); });
                var("r<2,256,5,4,8,3,SP> noY", [&] { if (run_dgradr<2, 256, 5, 4, 8, 3, 2>(b, st)) printf("    (n/a)\n"); });
                b.yact = a.yact;
            } else if (M == 32 && J == 3) {
                var("r<1,256,3,6,32>", [&] { if (run_dgradr<1, 256, 3, 6, 32>(b, st)) printf("    (n/a)\n"); });
                var("r<1,256,3,6,32,1,SP>", [&] { if (run_dgradr<1, 256, 3, 6, 32, 1, 2>(b, st)) printf("    (n/a)\n"); });
                var("r<1,256,3,6,16,2,SP>", [&] { if (run_dgradr<1, 256, 3, 6, 16, 2, 2>(b, st)) printf("    (n/a)\n"); });
            }
            tot_new[1] += best;
        }
        // ---- first-layer backward data (VALU kernel): element vs quad staging
        if (l.sf == 1 && l.KF == 9 && l.Ci == 2 && (!only || !strcmp(only, "dgrad"))) {
            C2Dg a{g, dy, yact, wp, nullptr, dx0, 0, 0, 0, 0, 0, 0};
            dim3 grid((unsigned)cdiv(l.Fi, DN_COLS), (unsigned)cdiv(l.T2, DN_ROWS), (unsigned)B);
            double t0 = time_ms([&] { hipLaunchKernelGGL((c2_dgrad_narrow<2, 3, 9, true, false>), grid, dim3(NT), 0, st, a); });
            printf("  dgrad narrow elem            %8.1f us  %6.1f TF/s\n", t0 * 1e3, flops / t0 * 1e-9);
            C2Dg b = a;
            b.dx = dx1;
            CK(hipMemset(dx1, 0, nx * 4));
            double t1 = time_ms([&] { hipLaunchKernelGGL((c2_dgrad_narrow<2, 3, 9, true, true>), grid, dim3(NT), 0, st, b); });
            double e = rel_err(dx1, dx0, nx);
            printf("  dgrad narrow quad            %8.1f us  %6.1f TF/s  err %.1e%s\n", t1 * 1e3, flops / t1 * 1e-9, e,
                   e > 1e-6 ? "  MISMATCH" : "");
            b.yact = nullptr;
            double t2 = time_ms([&] { hipLaunchKernelGGL((c2_dgrad_narrow<2, 3, 9, false, true>), grid, dim3(NT), 0, st, b); });
            printf("  dgrad narrow quad noY        %8.1f us  %6.1f TF/s\n", t2 * 1e3, flops / t2 * 1e-9);
        }
        // ---- weight grad (+ bias column)
        if (!only || !strcmp(only, "wgrad")) {
            const int N = l.Ci * l.KT * l.KF + 1;
            float* dw0 = dev_zero((size_t)l.Co * N);
            float* db0 = dev_zero(l.Co);
            float* dw1 = dev_zero((size_t)l.Co * N);
            float* db1 = dev_zero(l.Co);
            WgPlan2 p = plan_wg2(g);
            float* ws = dev_zero((size_t)(p.splits > 4096 ? p.splits : 4096) * l.Co * N);
            auto old = [&] {
                C2Wg a{g, dy, yact, x, ws, p.BT, p.NR, p.RL, p.NCmax, p.items, p.per_split, p.chunks};
                const size_t lds = ((size_t)4 * p.NCmax * p.NR + (size_t)p.BT * 32 + (size_t)p.NCmax * p.NR * p.RL) *
                                       sizeof(float) + p.BT * sizeof(int);
                if (p.narrow) {
                    const size_t red = (size_t)4 * 16 * 64 * sizeof(float);
                    hipLaunchKernelGGL((c2_wgrad_kernel<32, 64, 1, 2, 2>), dim3((unsigned)cdiv(N, 64), 1, p.splits),
                                       dim3(NT), lds > red ? lds : red, st, a);
                } else {
                    hipLaunchKernelGGL((c2_wgrad_kernel<32, 128, 1, 4, 1>), dim3((unsigned)cdiv(N, 128), 1, p.splits),
                                       dim3(NT), lds, st, a);
                }
                hipLaunchKernelGGL(c2_wg_reduce, dim3((unsigned)cdiv(l.Co * N, 64)), dim3(256), 0, st, ws, p.splits,
                                   l.Co, N, dw0, db0, 0, 0);
            };
            double t0 = time_ms(old);
            printf("  wgrad old                    %8.1f us  %6.1f TF/s\n", t0 * 1e3, flops / t0 * 1e-9);
            tot_old[2] += t0;
            double best = t0;
            const int gc = wg3_gc(g);
            auto var = [&](const char* nm, int target, std::function<void(const WgPlan3&)> f) {
                WgPlan3 q = plan_wg3(g, gc, target);
                CK(hipMemset(dw1, 0, (size_t)l.Co * N * 4));
                double t = time_ms([&] {
                    f(q);
                    hipLaunchKernelGGL(c2_wg_reduce, dim3((unsigned)cdiv(l.Co * N, 64)), dim3(256), 0, st, ws, q.splits,
                                       l.Co, N, dw1, db1, 0, 0);
                });
                double e = fmax(rel_err(dw1, dw0, (size_t)l.Co * (N - 1)), rel_err(db1, db0, l.Co));
                printf("  wgrad %-23s %8.1f us  %6.1f TF/s  err %.1e%s  (splits %d, lds %zu)\n", nm, t * 1e3,
                       flops / t * 1e-9, e, e > 1e-5 ? "  MISMATCH" : "", q.splits, q.lds);
                if (e <= 1e-5 && t < best) best = t;
            };
            auto var3 = [&](const char* nm, int gc3, int target, std::function<int(const WgPlan3&)> f) {
                WgPlan3 q = plan_wg3r(g, gc3, target);
                CK(hipMemset(dw1, 0, (size_t)l.Co * N * 4));
                bool bad = false;
                double t = time_ms([&] {
                    if (f(q)) bad = true;
                    hipLaunchKernelGGL(c2_wg_reduce, dim3((unsigned)cdiv(l.Co * N, 64)), dim3(256), 0, st, ws, q.splits,
                                       l.Co, N, dw1, db1, 0, 0);
                });
                if (bad) { printf("  wgrad %-23s n/a\n", nm); return; }
                double e = fmax(rel_err(dw1, dw0, (size_t)l.Co * (N - 1)), rel_err(db1, db0, l.Co));
                printf("  wgrad %-23s %8.1f us  %6.1f TF/s  err %.1e%s  (splits %d, lds %zu)\n", nm, t * 1e3,
                       flops / t * 1e-9, e, e > 1e-5 ? "  MISMATCH" : "", q.splits, q.lds);
                if (e <= 1e-5 && t < best) best = t;
            };
            if (wgr_ok(g)) {
                for (int waves : {1024, 1536, 2048}) {
                    const WgPlanR q = plan_wgr(g, waves);
                    CK(hipMemset(dw1, 0, (size_t)l.Co * N * 4));
                    double t = time_ms([&] {
                        run_wgrad_rw(g, dy, yact, x, ws, q, st);
                        hipLaunchKernelGGL(c2_wg_reduce, dim3((unsigned)cdiv(l.Co * N, 64)), dim3(256), 0, st, ws, q.splits,
                                           l.Co, N, dw1, db1, 0, 0);
                    });
                    double tk = time_ms([&] { run_wgrad_rw(g, dy, yact, x, ws, q, st); });
                    double e = fmax(rel_err(dw1, dw0, (size_t)l.Co * (N - 1)), rel_err(db1, db0, l.Co));
                    printf("  wgrad rw %-20d %8.1f us  %6.1f TF/s  err %.1e%s  (splits %d, kernel only %.1f us %.1f TF/s)\n",
                           waves, t * 1e3, flops / t * 1e-9, e, e > 1e-5 ? "  MISMATCH" : "", q.splits, tk * 1e3,
                           flops / tk * 1e-9);
                    if (e <= 1e-5 && t < best) best = t;
                }
            }
            if (gc && l.KF == 9) {
                var3("3<9,1,9,4,1,5,PF0> 768", 32, 768, [&](const WgPlan3& q) { return run_wgrad3<9, 1, 9, 4, 1, 5, 0>(g, dy, yact, x, ws, q, st); });
            } else if (l.Ci == 2 && l.KF == 9) {  // first layer: all 6 combos in one group, 54 of 64 columns
                var3("3<9,1,2,2,4,4> 6/768", 6, 768, [&](const WgPlan3& q) { return run_wgrad3<9, 1, 2, 2, 4, 4>(g, dy, yact, x, ws, q, st); });
                var3("3<9,1,2,2,4,8> 6/768", 6, 768, [&](const WgPlan3& q) { return run_wgrad3<9, 1, 2, 2, 4, 8>(g, dy, yact, x, ws, q, st); });
                var3("3<9,1,2,2,4,4> 6/1536", 6, 1536, [&](const WgPlan3& q) { return run_wgrad3<9, 1, 2, 2, 4, 4>(g, dy, yact, x, ws, q, st); });
                var3("3<9,2,1,4,8,4> 6/768", 6, 768, [&](const WgPlan3& q) { return run_wgrad3<9, 2, 1, 4, 8, 4>(g, dy, yact, x, ws, q, st); });
                var3("3<9,2,1,4,8,8> 6/1536", 6, 1536, [&](const WgPlan3& q) { return run_wgrad3<9, 2, 1, 4, 8, 8>(g, dy, yact, x, ws, q, st); });
                var3("3<9,1,2,2,4,4> 6/768 noY", 6, 768, [&](const WgPlan3& q) { return run_wgrad3<9, 1, 2, 2, 4, 4>(g, dy, nullptr, x, ws, q, st); });
            } else if (gc && l.KF == 3 && getenv("MB_L4_BN64")) {
                // the 3x3 layer on 64-column tiles (5 tiles for its 289 columns instead of 3 x 128)
                for (int tgt : {1024, 2048}) {
                    WgPlan2 p2 = plan_wg2(g);
                    p2.narrow = 1;
                    p2.NCmax = 63 / l.KF + 2;
                    const int tiles = (int)(cdiv(N, 64) * cdiv(l.Co, 32));
                    int sp = (int)cdiv(tgt, tiles);
                    if (sp > p2.items) sp = p2.items;
                    p2.per_split = (int)cdiv(p2.items, sp);
                    p2.splits = (int)cdiv(p2.items, p2.per_split);
                    C2Wg a2{g, dy, yact, x, ws, p2.BT, p2.NR, p2.RL, p2.NCmax, p2.items, p2.per_split, p2.chunks};
                    const size_t lds = ((size_t)4 * p2.NCmax * p2.NR + (size_t)p2.BT * 32 + (size_t)p2.NCmax * p2.NR * p2.RL) *
                                           sizeof(float) + p2.BT * sizeof(int);
                    const size_t red = (size_t)4 * 16 * 64 * sizeof(float);
                    CK(hipMemset(dw1, 0, (size_t)l.Co * N * 4));
                    double t = time_ms([&] {
                        hipLaunchKernelGGL((c2_wgrad_kernel<32, 64, 1, 2, 2>), dim3((unsigned)cdiv(N, 64), 1, p2.splits),
                                           dim3(NT), lds > red ? lds : red, st, a2);
                        hipLaunchKernelGGL(c2_wg_reduce, dim3((unsigned)cdiv(l.Co * N, 64)), dim3(256), 0, st, ws, p2.splits,
                                           l.Co, N, dw1, db1, 0, 0);
                    });
                    double e = fmax(rel_err(dw1, dw0, (size_t)l.Co * (N - 1)), rel_err(db1, db0, l.Co));
                    printf("  wgrad <32,64,1,2,2> %d      %8.1f us  %6.1f TF/s  err %.1e%s  (splits %d)\n", tgt, t * 1e3,
                           flops / t * 1e-9, e, e > 1e-5 ? "  MISMATCH" : "", p2.splits);
                }
            } else if (gc && l.KF == 3) {
                var3("3<3,1,9,16,1,1,PF0> 96/512", 96, 512, [&](const WgPlan3& q) { return run_wgrad3<3, 1, 9, 16, 1, 1, 0>(g, dy, yact, x, ws, q, st); });
                var3("3<3,1,9,16,1,1,PF1> 96/512", 96, 512, [&](const WgPlan3& q) { return run_wgrad3<3, 1, 9, 16, 1, 1, 1>(g, dy, yact, x, ws, q, st); });
                var3("3<3,1,9,16,1,2,PF1> 96/768", 96, 768, [&](const WgPlan3& q) { return run_wgrad3<3, 1, 9, 16, 1, 2, 1>(g, dy, yact, x, ws, q, st); });
                var3("3<3,3,3,24,3,1,PF1> 96/512", 96, 512, [&](const WgPlan3& q) { return run_wgrad3<3, 3, 3, 24, 3, 1, 1>(g, dy, yact, x, ws, q, st); });
                var3("3<3,3,3,24,3,2,PF1> 96/768", 96, 768, [&](const WgPlan3& q) { return run_wgrad3<3, 3, 3, 24, 3, 2, 1>(g, dy, yact, x, ws, q, st); });
            }
            tot_new[2] += best;
            CK(hipFree(dw0)); CK(hipFree(db0)); CK(hipFree(dw1)); CK(hipFree(db1)); CK(hipFree(ws));
        }
        CK(hipFree(x)); CK(hipFree(wf)); CK(hipFree(bias)); CK(hipFree(y0)); CK(hipFree(y1)); CK(hipFree(dy));
        CK(hipFree(yact)); CK(hipFree(dx0)); CK(hipFree(dx1)); CK(hipFree(wp));
    }
    printf("\nsum over layers (one call each), ms: fwd %.3f -> %.3f, dgrad %.3f -> %.3f, wgrad %.3f -> %.3f\n",
           tot_old[0], tot_new[0], tot_old[1], tot_new[1], tot_old[2], tot_new[2]);
    return 0;
}
