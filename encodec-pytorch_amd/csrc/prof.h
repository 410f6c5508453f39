// In-library launch timing for bench.py's roofline line (encx_prof_enable / encx_prof_read).
// When enabled, each public MFMA entry point brackets its launches with a hipEvent pair on the
// caller's stream and books its algorithmic FLOPs / bytes. Disabled: one branch, no events.
// timed = false books the FLOPs / bytes only (no events): the small elementwise / reduction
// entry points, so the whole-step algorithmic totals are complete without paying an event
// pair per tiny launch.
#pragma once
#include <hip/hip_runtime.h>

struct encx_prof_scope {
    hipStream_t st;
    int slot;
    encx_prof_scope(hipStream_t s, double flops, double bytes, const char* kind = "", bool timed = true);
    ~encx_prof_scope();
    // per-launch label (shape) for the per-slot table; printf-style, only formatted when on
    void tag(const char* fmt, ...);
};
