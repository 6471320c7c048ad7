// rt_knobs.cpp — the library's RT580_* environment switches, validated in one
// place (rt_gpu_init). Each switch is read where it acts (rt_shim.cpp,
// rt_kernels.hip, rt_bvh.cpp, raytracer.cpp); this table is the contract: a
// variable named RT580_* that is not listed, or whose value is outside its
// set, makes rt_gpu_init fail with RT_FAILURE instead of being ignored or
// half-applied. Defaults are the measured product settings (DESIGN.md,
// INTEGRATION.md lists every switch).
#include "rt_knobs.h"

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

extern char** environ;

namespace rt580 {
namespace {

enum Kind { INT_SET, INT_RANGE, STRING_SET, NOT_LIBRARY, DIAG_ONLY };

struct Knob {
    const char* name;
    Kind kind;
    long lo, hi;          // INT_RANGE bounds
    const long* set;      // INT_SET values (terminated by -1)
    const char* const* strs;  // STRING_SET values (null-terminated)
};

const long k01[] = {0, 1, -1};
const long k234[] = {2, 3, 4, -1};
const char* const kTransport[] = {"rccl", "local", nullptr};

// Every product switch selects a behaviour of the library, not a kernel form:
// the forms measured slower in earlier rounds were removed with their switches
// (DESIGN.md "Measured and rejected"). tests/test_knobs.py exercises each one.
const Knob kKnobs[] = {
    // rt_shim.cpp / raytracer.cpp
    {"RT580_PIPELINE", INT_SET, 0, 0, k01, nullptr},        // 0: every frame on the caller's stream
    {"RT580_SLOTS", INT_SET, 0, 0, k234, nullptr},          // frames in flight
    {"RT580_AO_ORDER", INT_SET, 0, 0, k01, nullptr},        // 1: AO phases of consecutive frames in order
    {"RT580_CHUNK_LOG2", INT_RANGE, 6, 27, nullptr, nullptr},  // largest far-queue / AO-ray chunk (rays)
    {"RT580_GRID_COARSE_PX", INT_RANGE, 0, 1L << 31, nullptr, nullptr},  // frames below: the half-resolution grid
    {"RT580_MULTI_TRANSPORT", STRING_SET, 0, 0, nullptr, kTransport},
    {"RT580_GPUS", INT_RANGE, 1, 16, nullptr, nullptr},     // Render()'s GPU count
    {"RT580_REPLAY", INT_SET, 0, 0, k01, nullptr},          // 0: BVH frames read their counts on the host
    {"RT580_GRAPH", INT_SET, 0, 0, k01, nullptr},           // 0: no HIP graph for Render()'s small frames
    {"RT580_D2H_MAPPED", INT_SET, 0, 0, k01, nullptr},      // 0: rank 0's PPM body through a device stage
    {"RT580_PROGRESS", INT_SET, 0, 0, k01, nullptr},        // a stderr line per BVH trace level / AO chunk
    // diagnostic builds (make diag) only
    {"RT580_BVH_DIAG", DIAG_ONLY, 0, 0, nullptr, nullptr},
    {"RT580_DUMP_FAR", DIAG_ONLY, 0, 0, nullptr, nullptr},
    {"RT580_REPLAY_CORRUPT", DIAG_ONLY, 0, 0, nullptr, nullptr},
    {"RT580_CELL_SKIP", DIAG_ONLY, 0, 0, nullptr, nullptr},
    {"RT580_AO_VERIFY", DIAG_ONLY, 0, 0, nullptr, nullptr},
    // read by the Python binding and the tests, not by the library
    {"RT580_LIB", NOT_LIBRARY, 0, 0, nullptr, nullptr},
    {"RT580_EXHAUSTIVE", NOT_LIBRARY, 0, 0, nullptr, nullptr},
};

bool parse_long(const char* v, long& out) {
    if (!*v) return false;
    char* end = nullptr;
    errno = 0;
    out = std::strtol(v, &end, 10);
    return errno == 0 && end && *end == '\0';
}

// "" when the value is valid, else why not
std::string check(const Knob& k, const char* v) {
    long n = 0;
    switch (k.kind) {
        case INT_SET:
            if (!parse_long(v, n)) return "not an integer";
            for (const long* p = k.set; *p >= 0; p++)
                if (*p == n) return "";
            return "not one of the supported values";
        case INT_RANGE:
            if (!parse_long(v, n)) return "not an integer";
            if (n < k.lo || n > k.hi)
                return "outside [" + std::to_string(k.lo) + ", " + std::to_string(k.hi) + "]";
            return "";
        case STRING_SET:
            for (const char* const* p = k.strs; *p; p++)
                if (!std::strcmp(*p, v)) return "";
            return "not one of the supported values";
        case DIAG_ONLY:
#ifdef RT580_DIAGNOSTICS
            return "";
#else
            return "read by diagnostic builds only (make diag)";
#endif
        case NOT_LIBRARY:
            return "";
    }
    return "";
}

}  // namespace

bool knobs_check(char* err, size_t n) {
    for (char** e = environ; e && *e; e++) {
        if (std::strncmp(*e, "RT580_", 6) != 0) continue;
        const char* eq = std::strchr(*e, '=');
        if (!eq) continue;
        const std::string name(*e, (size_t)(eq - *e));
        const Knob* k = nullptr;
        for (const Knob& c : kKnobs)
            if (name == c.name) k = &c;
        if (!k) {
            std::snprintf(err, n, "unknown environment switch %s (INTEGRATION.md lists the RT580_* switches)",
                          name.c_str());
            return false;
        }
        const std::string why = check(*k, eq + 1);
        if (!why.empty()) {
            std::snprintf(err, n, "%s=%s: %s", name.c_str(), eq + 1, why.c_str());
            return false;
        }
    }
    return true;
}

}  // namespace rt580
