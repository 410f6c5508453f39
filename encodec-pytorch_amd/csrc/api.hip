// Library entry points: version, error strings, device selection, launch profiling.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>

#include "common.h"
#include "prof.h"

namespace {
constexpr int kMaxSlots = 1 << 14;
struct ProfState {
    std::mutex mu;
    bool on = false;
    int next = 0;
    hipEvent_t ev0[kMaxSlots];
    hipEvent_t ev1[kMaxSlots];
    double flops[kMaxSlots];
    double bytes[kMaxSlots];
    bool timed[kMaxSlots];
    char tags[kMaxSlots][64];
    bool created = false;
};
ProfState g_prof;
std::atomic<bool> g_prof_on{false};

// kernel-selection options (common.h EncxOpt): id, name, default; initial value from ENCX_<name>
struct OptDef {
    EncxOpt id;
    const char* name;
    int64_t def;
};
constexpr OptDef kOpts[OPT_COUNT] = {
    {OPT_FFT, "FFT", 1}, {OPT_PW, "PW", 1}, {OPT_PW_TMAX, "PW_TMAX", 1024}, {OPT_PW_WG_TMAX, "PW_WG_TMAX", 12000}, {OPT_LSTM_FUSE, "LSTM_FUSE", 0},
    {OPT_LSTM_PERSIST, "LSTM_PERSIST", 1},
    {OPT_LSTM_WG_SPLITS, "LSTM_WG_SPLITS", 32},
    {OPT_FWR, "FWR", 256}, {OPT_DGR, "DGR", 256}, {OPT_WGR, "WGR", 2048},
    {OPT_WGR_WGS, "WGR_WGS", 256}, {OPT_FEAT_CODE, "FEAT_CODE", 1}, {OPT_CONV_CK, "CONV_CK", 64},
    {OPT_CONV_SPLIT, "CONV_SPLIT", 1024}, {OPT_CONV_WG_SPLIT, "CONV_WG_SPLIT", 1024},
    {OPT_CONV2, "CONV2", 7}, {OPT_CONV2_TILE, "CONV2_TILE", 0}, {OPT_CONV2_RED, "CONV2_RED", 64},
    {OPT_CONV2_KS, "CONV2_KS", 0}, {OPT_CONV2_WGS, "CONV2_WGS", 512},
    {OPT_CONV2_LOWT, "CONV2_LOWT", 0},
    {OPT_LSTM_SPIN, "LSTM_SPIN", 0}, {OPT_LSTM_FAULT, "LSTM_FAULT", 0},
    {OPT_BLAS, "BLAS", 3},
};
constexpr bool opts_in_order() {
    for (int i = 0; i < OPT_COUNT; ++i)
        if (kOpts[i].id != i) return false;
    return true;
}
static_assert(opts_in_order(), "kOpts must list every EncxOpt in enum order");
std::atomic<int64_t> g_opt[OPT_COUNT];
std::once_flag g_opt_once;
void opt_init() {
    std::call_once(g_opt_once, [] {
        for (int i = 0; i < OPT_COUNT; ++i) {
            char env[64];
            snprintf(env, sizeof(env), "ENCX_%s", kOpts[i].name);
            const char* v = getenv(env);
            g_opt[i].store(v ? atoll(v) : kOpts[i].def);
        }
    });
}
int opt_find(const char* name) {
    if (!name) return -1;
    if (!strncmp(name, "ENCX_", 5)) name += 5;
    for (int i = 0; i < OPT_COUNT; ++i)
        if (!strcmp(name, kOpts[i].name)) return i;
    return -1;
}
}  // namespace

int64_t encx_opt(EncxOpt id) {
    opt_init();
    return g_opt[id].load(std::memory_order_relaxed);
}

encx_prof_scope::encx_prof_scope(hipStream_t s, double f, double b, const char* kind, bool timed)
    : st(s), slot(-1) {
    if (!g_prof_on.load(std::memory_order_relaxed)) return;
    std::lock_guard<std::mutex> g(g_prof.mu);
    if (!g_prof.on || g_prof.next >= kMaxSlots) return;
    slot = g_prof.next++;
    g_prof.flops[slot] = f;
    g_prof.bytes[slot] = b;
    g_prof.timed[slot] = timed;
    snprintf(g_prof.tags[slot], sizeof(g_prof.tags[slot]), "%s", kind ? kind : "");
    if (timed) (void)hipEventRecord(g_prof.ev0[slot], st);
}

void encx_prof_scope::tag(const char* fmt, ...) {
    if (slot < 0) return;
    char* t = g_prof.tags[slot];
    size_t n = strlen(t);
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(t + n, sizeof(g_prof.tags[slot]) - n, fmt, ap);
    va_end(ap);
}

encx_prof_scope::~encx_prof_scope() {
    if (slot >= 0 && g_prof.timed[slot]) (void)hipEventRecord(g_prof.ev1[slot], st);
}

extern "C" {

int encx_version(void) { return 1; }

const char* encx_strerror(int code) {
    if (code == ENCX_OK) return "ok";
    if (code == ENCX_EINVAL) return "encx: invalid argument (shape, stride or null pointer)";
    return hipGetErrorString((hipError_t)code);
}

int encx_option_count(void) { return OPT_COUNT; }

const char* encx_option_name(int i) { return i >= 0 && i < OPT_COUNT ? kOpts[i].name : nullptr; }

int encx_get_option(const char* name, int64_t* value) {
    const int i = opt_find(name);
    if (i < 0 || !value) return ENCX_EINVAL;
    *value = encx_opt((EncxOpt)i);
    return 0;
}

int encx_set_option(const char* name, int64_t value, int64_t* previous) {
    const int i = opt_find(name);
    if (i < 0) return ENCX_EINVAL;
    opt_init();
    const int64_t prev = g_opt[i].exchange(value);
    if (previous) *previous = prev;
    return 0;
}

int encx_init(int device) {
    hipError_t e = hipSetDevice(device);
    return (int)e;
}

int encx_prof_enable(int on) {
    std::lock_guard<std::mutex> g(g_prof.mu);
    if (on && !g_prof.created) {
        // timing-only events: no system-scope fence on record, so bracketing a launch does not
        // write back and invalidate L2 (which would slow the kernels being measured)
        for (int i = 0; i < kMaxSlots; ++i) {
            if (hipEventCreateWithFlags(&g_prof.ev0[i], hipEventDisableSystemFence) != hipSuccess) return ENCX_EINVAL;
            if (hipEventCreateWithFlags(&g_prof.ev1[i], hipEventDisableSystemFence) != hipSuccess) return ENCX_EINVAL;
        }
        g_prof.created = true;
    }
    g_prof.on = on != 0;
    g_prof.next = 0;
    g_prof_on.store(g_prof.on);
    return 0;
}

int encx_prof_enabled(void) { return g_prof_on.load() ? 1 : 0; }

int encx_prof_read(double* total_ms, double* total_flops, double* total_bytes, int64_t* launches) {
    std::lock_guard<std::mutex> g(g_prof.mu);
    double ms = 0, fl = 0, by = 0;
    for (int i = 0; i < g_prof.next; ++i) {
        fl += g_prof.flops[i];
        by += g_prof.bytes[i];
        if (!g_prof.timed[i]) continue;
        hipError_t e = hipEventSynchronize(g_prof.ev1[i]);
        if (e != hipSuccess) return (int)e;
        float t = 0.f;
        e = hipEventElapsedTime(&t, g_prof.ev0[i], g_prof.ev1[i]);
        if (e != hipSuccess) return (int)e;
        ms += t;
    }
    if (total_ms) *total_ms = ms;
    if (total_flops) *total_flops = fl;
    if (total_bytes) *total_bytes = by;
    if (launches) *launches = g_prof.next;
    return 0;
}

int encx_prof_slot(int64_t i, double* ms, double* flops, double* bytes, const char** tag) {
    std::lock_guard<std::mutex> g(g_prof.mu);
    if (i < 0 || i >= g_prof.next) return ENCX_EINVAL;
    float t = -1.f;  // untimed (booked-only) slot
    if (g_prof.timed[i]) {
        hipError_t e = hipEventSynchronize(g_prof.ev1[i]);
        if (e != hipSuccess) return (int)e;
        e = hipEventElapsedTime(&t, g_prof.ev0[i], g_prof.ev1[i]);
        if (e != hipSuccess) return (int)e;
    }
    if (ms) *ms = t;
    if (flops) *flops = g_prof.flops[i];
    if (bytes) *bytes = g_prof.bytes[i];
    if (tag) *tag = g_prof.tags[i];
    return 0;
}

}  // extern "C"
