// rmat.hpp — deterministic Graph500-parameter RMAT generator, identical on host and
// device (counter-based hashing; integer quadrant thresholds; Feistel label bijection).
#pragma once
#include <cstdint>

#ifndef __HIPCC__
#define SHEEP_HD inline
#else
#define SHEEP_HD __host__ __device__ inline
#endif

namespace sheep {

struct RmatParams {
  int scale = 0;
  int half = 0;          // Feistel half width in bits: ceil(scale/2)
  uint64_t seed = 0;
  uint32_t tA = 0, tAB = 0, tABC = 0;   // cumulative quadrant thresholds on 32-bit draws
  uint64_t key[4] = {0, 0, 0, 0};
};

SHEEP_HD uint64_t mix64(uint64_t z) {   // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

inline RmatParams rmat_params(int scale, uint64_t seed) {
  RmatParams p;
  p.scale = scale;
  p.half = (scale + 1) / 2;
  p.seed = seed;
  const double A = 0.57, B = 0.19, C = 0.19;   // D = 0.05
  const double two32 = 4294967296.0;
  p.tA = (uint32_t)(A * two32);
  p.tAB = (uint32_t)((A + B) * two32);
  p.tABC = (uint32_t)((A + B + C) * two32);
  for (int r = 0; r < 4; ++r) p.key[r] = mix64(seed * 0x632BE59BD9B4E019ull + 0x1000 + r);
  return p;
}

// Bijection on [0, 2^scale): 4-round Feistel on 2*half bits with cycle walking.
SHEEP_HD uint32_t rmat_permute(uint32_t x, const RmatParams &p) {
  const uint32_t hm = (1u << p.half) - 1u;
  const uint64_t lim = 1ull << p.scale;
  do {
    uint32_t L = x >> p.half, R = x & hm;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      uint32_t F = (uint32_t)mix64((uint64_t)R ^ p.key[r]) & hm;
      uint32_t nL = R, nR = L ^ F;
      L = nL; R = nR;
    }
    x = (L << p.half) | R;
  } while ((uint64_t)x >= lim);
  return x;
}

// Edge i (0 <= i < ef << scale): quadrant walk, then label permutation.
SHEEP_HD void rmat_edge(uint64_t i, const RmatParams &p, uint32_t &u, uint32_t &v) {
  uint32_t a = 0, b = 0;
  for (int l = 0; l < p.scale; l += 2) {
    uint64_t r = mix64(p.seed ^ ((i << 5) | (uint64_t)(l >> 1)) * 0xD1B54A32D192ED03ull);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (l + k >= p.scale) break;
      uint32_t d = (uint32_t)(r >> (32 * k));
      uint32_t ub = d >= p.tAB ? 1u : 0u;                               // C or D
      uint32_t vb = (d >= p.tA && d < p.tAB) || d >= p.tABC ? 1u : 0u;  // B or D
      a |= ub << (l + k);
      b |= vb << (l + k);
    }
  }
  u = rmat_permute(a, p);
  v = rmat_permute(b, p);
}

// Sort/dedup key: tail = max, head = min (orientation of data/hep-th.dat).
SHEEP_HD uint64_t rmat_key(uint32_t u, uint32_t v, int scale) {
  uint32_t t = u > v ? u : v, h = u > v ? v : u;
  return ((uint64_t)t << scale) | h;
}

}  // namespace sheep
