// Raytracer.h — drop-in replacement for the reference's "580 Raytracer/Raytracer.h":
// a caller written against the reference (e.g. its main(), Raytracer.cpp:944-953)
// compiles unchanged against this header and links lib580rt.so; Render() then
// runs the per-pixel path on the GPU(s). See INTEGRATION.md.
#pragma once
#include "../580-raytracer_amd/csrc/raytracer.h"
