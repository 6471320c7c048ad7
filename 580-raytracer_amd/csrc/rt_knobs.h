// rt_knobs.h — validation of the RT580_* environment switches (rt_knobs.cpp).
#pragma once
#include <stddef.h>

namespace rt580 {
// Every RT580_* variable of the environment is a known switch with a valid
// value; otherwise false and the reason in err.
bool knobs_check(char* err, size_t n);
}  // namespace rt580
