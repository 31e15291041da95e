// tree_tour.hpp — kid table + Euler tour of an elimination forest (device resident).
#pragma once
#include "common.hpp"

struct sheep_kids {
  sheep::Ctx *ctx = nullptr;
  uint64_t n = 0;
  uint32_t *parent = nullptr;  // copy of the tree's parent array
  uint32_t *koff = nullptr;    // n+1 offsets into kids
  uint32_t *kids = nullptr;    // child lists, initially ascending id (jnode.h:190-204);
                               // FFD sorts segments in place (persistent, partition.cpp:104-106)
  uint32_t *kpar = nullptr;    // kpar[i] = the parent whose list holds kids[i] (the sorted keys)
  uint64_t nkids = 0;
  uint64_t max_kids = 0;       // the largest kid count
  uint64_t cap = 0;            // the buffers hold cap + 2 / cap + 1 words
};

namespace sheep {

// Euler tour positions of every non-root node's down arc (tD) and up arc (tU) in one
// list that chains the tours of the roots with kids in ascending root id.
struct Tour {
  uint64_t A = 0;              // number of arcs = 2 * (n - roots)
  uint32_t *tD = nullptr, *tU = nullptr;
  uint32_t *rk = nullptr;      // roots with kids, ascending
  uint64_t nrk = 0;
  uint64_t nroots = 0;
};

void build_kids(Ctx &c, const sheep_jnode *tree, uint64_t n, sheep_kids *k);
void release_kids(Ctx *c, sheep_kids *k);
void build_tour(Ctx &c, sheep_kids *k, Tour &t);
// generic helpers
void gather_u32(Ctx &c, const uint32_t *src, const uint32_t *idx, uint64_t m, uint32_t *dst);

}  // namespace sheep
