// rt_mt.h — block jump-ahead of MSVC's default_random_engine (std::mt19937,
// the reference's member mGenerator, Raytracer.h:592; draws consumed by
// RandomUnitVector, Raytracer.cpp:269-281) so that the device can generate any
// window of the serial stream in parallel (rt_kernels.hip mt_generate_kernel)
// instead of the host generating every draw before it.
//
// The engine's raw words y_0, y_1, ... obey y_{n+624} = y_{n+397} ^ f(y_n,
// y_{n+1}) (the twist), draw k is temper(y_{624+k}), and W_n = (y_n .. y_{n+623})
// is a state from which the twist produces the draws n, n+1, ... The one-word
// shift A: W_n -> W_{n+1} is GF(2)-linear with minimal polynomial x phi(x),
// phi the engine's degree-19937 characteristic polynomial (the factor x: the
// low 31 bits of y_n never reach a later word), so for J >= 1
//     W_{n+J} = A h(A) W_n,   h = x^(J-1) mod phi,
// evaluated by Horner's rule with A as one twist step of a 624-word ring.
// phi comes from the Berlekamp-Massey algorithm on 2 x 19937 output bits.
// Checked against std::mt19937 itself (tests/native/mt_check.cpp).
#pragma once
#include <stdint.h>

#include <vector>

namespace rt580 {

constexpr int kMtN = 624;
// Draws per checkpoint block of the device generator: a multiple of 624.
constexpr uint64_t kMtBlock = 624ull * 4096ull;

struct MtWindow {
    uint32_t y[kMtN];  // W_n: y_n .. y_{n+623}; the twist of it gives draws n .. n+623
};

// W_0 of std::mt19937(seed) (its state right after seeding).
MtWindow mt_seed_window(uint32_t seed);
// W_{n+J} from W_n (J >= 0). Cost: one polynomial x^(J-1) mod phi (~36 modular
// squarings for J ~ 2^36) and one Horner evaluation (~19937 twist steps).
MtWindow mt_jump(const MtWindow& w, uint64_t J);
// The windows W_{k kMtBlock} for k in [k0, k1) of the stream of `seed`, copied
// into `out`, from a process-wide cache (one run of consecutive windows per
// seed, under a lock: computed on demand in parallel from one jump to its
// first window, extended or restarted by later calls). False if the engine's
// polynomial could not be found.
bool mt_checkpoints(uint32_t seed, uint64_t k0, uint64_t k1, std::vector<MtWindow>& out);
// Host reference: draws [n, n + count) from W_n by the twist (tests).
void mt_draws(const MtWindow& w, uint64_t count, uint32_t* out);

}  // namespace rt580
