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

enum Kind { INT_SET, INT_RANGE, FLOAT_NONNEG, FLOAT_POS, STRING_SET, NOT_LIBRARY, DIAG_ONLY };

struct Knob {
    const char* name;
    Kind kind;
    long lo, hi;          // INT_RANGE bounds
    const long* set;      // INT_SET values (terminated by -1)
    const char* const* strs;  // STRING_SET values (null-terminated)
};

const long k01[] = {0, 1, -1};
const long k23[] = {2, 3, -1};
const long k234[] = {2, 3, 4, -1};
const long kSort[] = {0, 1, 2, 3, -1};
const long kTraceWpe[] = {4, 6, 7, 8, -1};
const long kNearWpe[] = {0, 5, 6, 8, -1};
const long kLateWpe[] = {6, 8, -1};
const long kFarMode[] = {0, 1, 2, 3, 4, -1};
const long kFarU[] = {1, 2, 4, -1};
const long kFarCU[] = {0, 1, 2, 4, -1};
const long k0123[] = {0, 1, 2, 3, -1};
const long k148[] = {1, 4, 8, -1};
const long kSmallWpe[] = {0, 5, 6, -1};
// the AO kernel flavours launch_ao_small instantiates (rt_kernels.hip)
const long kAoVariant[] = {
    0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,                            // ao_kernel<v>
    1032, 3080, 3084, 7176, 7180, 7182,                                               // ao_kernel<v>, v >= 32
    16 | 1, 16 | 9, 16 | 8, 16 | 1032, 16 | 2056, 16 | 3080, 16 | 3084, 16 | 7176,   // ao_kernel_occ8<v>
    16 | 5128, 16 | 7180, 16 | 7182,
    32768 | 7180, 32768 | 16 | 7180,                                                  // two samples per lane
#ifdef RT580_DIAGNOSTICS
    41, 73, 105, 137, 233,
#endif
    -1};
const char* const kTransport[] = {"rccl", "local", nullptr};

const Knob kKnobs[] = {
    // rt_shim.cpp / raytracer.cpp
    {"RT580_PIPELINE", INT_SET, 0, 0, k01, nullptr},
    {"RT580_PHASE_EVENTS", INT_SET, 0, 0, k01, nullptr},
    {"RT580_SLOTS", INT_SET, 0, 0, k234, nullptr},
    {"RT580_AO_ORDER", INT_SET, 0, 0, k01, nullptr},
    {"RT580_SMALL_SLOTS", INT_SET, 0, 0, k234, nullptr},
    {"RT580_CHUNK_LOG2", INT_RANGE, 6, 27, nullptr, nullptr},
    {"RT580_GRID_LOG2", INT_RANGE, 0, 12, nullptr, nullptr},
    {"RT580_GRID_COARSE_PX", INT_RANGE, 0, 1L << 31, nullptr, nullptr},
    {"RT580_BVH4", INT_SET, 0, 0, k01, nullptr},
    {"RT580_CALL_HINT", INT_SET, 0, 0, k01, nullptr},
    {"RT580_MULTI_TRANSPORT", STRING_SET, 0, 0, nullptr, kTransport},
    {"RT580_GPUS", INT_RANGE, 1, 16, nullptr, nullptr},
    {"RT580_REPLAY", INT_SET, 0, 0, k01, nullptr},
    {"RT580_GRAPH", INT_SET, 0, 0, k01, nullptr},
    {"RT580_LAT_SPLIT_PCT", INT_RANGE, 1, 99, nullptr, nullptr},
    // rt_bvh.cpp
    {"RT580_LEAF_MAX", INT_RANGE, 1, 8, nullptr, nullptr},
    {"RT580_BVH_INFLATE", FLOAT_NONNEG, 0, 0, nullptr, nullptr},
    {"RT580_GRID_R", FLOAT_POS, 0, 0, nullptr, nullptr},
    // rt_kernels.hip
    {"RT580_AO_SPLIT", INT_SET, 0, 0, k01, nullptr},
    {"RT580_NEAR_WAVE", INT_SET, 0, 0, k01, nullptr},
    {"RT580_TRACE_LDS", INT_SET, 0, 0, k01, nullptr},
    {"RT580_AO_SORT", INT_SET, 0, 0, kSort, nullptr},
    {"RT580_AO_BUDGET", INT_RANGE, 0, 64, nullptr, nullptr},
    {"RT580_AO_BUDGET2", INT_SET, 0, 0, k01, nullptr},
    {"RT580_AO_RESUME", INT_SET, 0, 0, k01, nullptr},
    {"RT580_D2H_MAPPED", INT_SET, 0, 0, k01, nullptr},
    {"RT580_SMALL_TRACE_WPE", INT_SET, 0, 0, kSmallWpe, nullptr},
    {"RT580_TRACE_SPEC", INT_SET, 0, 0, k0123, nullptr},
    {"RT580_AO_SPEC", INT_RANGE, 0, 31, nullptr, nullptr},
    {"RT580_AO_REFILL", INT_RANGE, 0, 3, nullptr, nullptr},
    {"RT580_AO_REFILL_MIN", INT_RANGE, 1, 64, nullptr, nullptr},
    {"RT580_SMALL_SORT", INT_SET, 0, 0, k01, nullptr},
    {"RT580_D2H_BLOCKS", INT_RANGE, 1, 65536, nullptr, nullptr},
    {"RT580_TRACE_WPE", INT_SET, 0, 0, kTraceWpe, nullptr},
    {"RT580_NEAR_WPE", INT_SET, 0, 0, kNearWpe, nullptr},
    {"RT580_LATE_WPE", INT_SET, 0, 0, kLateWpe, nullptr},
    {"RT580_BRUTE_SPLIT", INT_SET, 0, 0, k0123, nullptr},
    {"RT580_BRUTE_RAYS", INT_SET, 0, 0, k148, nullptr},
    {"RT580_BRUTE_WAVES", INT_RANGE, 256, 1 << 20, nullptr, nullptr},
    {"RT580_FAR_MODE", INT_SET, 0, 0, kFarMode, nullptr},
    {"RT580_FAR_U", INT_SET, 0, 0, kFarU, nullptr},
    {"RT580_FAR_CLOSEST_U", INT_SET, 0, 0, kFarCU, nullptr},
    {"RT580_SORT_BITS", INT_SET, 0, 0, k01, nullptr},
    {"RT580_DEEP_GRID", INT_RANGE, 64, 65536, nullptr, nullptr},
    {"RT580_AO_GRID", INT_RANGE, 256, 1 << 20, nullptr, nullptr},
    {"RT580_AO_VARIANT", INT_SET, 0, 0, kAoVariant, nullptr},
    {"RT580_TRACE_SCALAR", INT_SET, 0, 0, k01, nullptr},
    {"RT580_RESOLVE", INT_SET, 0, 0, k01, nullptr},
    {"RT580_XCD_ORDER", INT_SET, 0, 0, k01, nullptr},
    {"RT580_PROGRESS", INT_SET, 0, 0, k01, nullptr},
    // diagnostic builds (make diag) only
    {"RT580_BVH_DIAG", DIAG_ONLY, 0, 0, nullptr, nullptr},
    {"RT580_DUMP_FAR", DIAG_ONLY, 0, 0, nullptr, nullptr},
    {"RT580_REPLAY_CORRUPT", DIAG_ONLY, 0, 0, nullptr, nullptr},
    {"RT580_CELL_SKIP", DIAG_ONLY, 0, 0, nullptr, nullptr},
    {"RT580_AO_VERIFY", DIAG_ONLY, 0, 0, nullptr, nullptr},
    {"RT580_LATE_REREAD", DIAG_ONLY, 0, 0, nullptr, nullptr},
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

bool parse_double(const char* v, double& out) {
    if (!*v) return false;
    char* end = nullptr;
    errno = 0;
    out = std::strtod(v, &end);
    return errno == 0 && end && *end == '\0' && std::isfinite(out);
}

// "" when the value is valid, else why not
std::string check(const Knob& k, const char* v) {
    long n = 0;
    double x = 0;
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
        case FLOAT_NONNEG:
            if (!parse_double(v, x) || x < 0) return "not a finite number >= 0";
            return "";
        case FLOAT_POS:
            if (!parse_double(v, x) || !(x > 0)) return "not a finite number > 0";
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
