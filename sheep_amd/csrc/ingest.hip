// ingest.hip — .net (SNAP text) edge lists parsed on the GPU.
//
// The reference reads .net files two ways: LLAMA's text loader for the graph
// (graph_wrapper.h:43-63; un-vendored) and SNAPReader for file sequences and the
// file-order partition writer (readerwriter.h:78-90): `stream >> X` then `stream >> Y`,
// stopping at the first pair that does not parse.  Here the text is uploaded once and
// parsed in parallel, byte-bound:
//   1. token starts (a non-blank byte after a blank one) counted per 4 KiB tile, scanned;
//   2. token start offsets written in order;
//   3. every token parsed the way istream >> reads an unsigned int, or "bad"; whether a
//      newline precedes it (a line's first token); whether it opens a comment line;
//   4. with skip_comments (the graph loader) tokens on '#' / '%' lines are dropped (line
//      ids by a scan of the line-start flags); the first bad token left ends the input,
//      as SNAPReader's failed >> does, and the valid tokens before it pair up into
//      records {tail, head, 1.0f} (an incomplete last pair is dropped).
// Tokens are read as istream >> reads an unsigned int (signs, wrap-around, leading zeros,
// a number followed by other characters: k_tok_parse); pinned by the reference's own
// SNAPReader on tests/golden/snap_cases.json.  Not followed: a token that holds two
// numbers glued by a sign ("4-5": istream reads 4 and then -5) ends the input after 4.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include "common.hpp"

namespace sheep {
namespace {

constexpr int NB_PER = 16;                  // bytes per thread
constexpr int NB_TILE = BLOCK * NB_PER;     // 4 KiB per workgroup tile

__device__ __forceinline__ bool blank(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

__device__ __forceinline__ bool tok_start(const char *text, uint64_t i) {
  return !blank(text[i]) && (i == 0 || blank(text[i - 1]));
}

__global__ __launch_bounds__(BLOCK) void k_tok_count(const char *__restrict__ text, uint64_t bytes,
                                                     uint32_t *__restrict__ tcnt) {
  const uint64_t base = (uint64_t)blockIdx.x * NB_TILE + (uint64_t)threadIdx.x * NB_PER;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < NB_PER; ++j)
    if (base + j < bytes && tok_start(text, base + j)) ++c;
  c = wave_sum(c);
  __shared__ uint32_t s[BLOCK / WAVE];
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tcnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ __launch_bounds__(BLOCK) void k_tok_write(const char *__restrict__ text, uint64_t bytes,
                                                     const uint32_t *__restrict__ toff, uint64_t *__restrict__ tpos) {
  const uint64_t base = (uint64_t)blockIdx.x * NB_TILE + (uint64_t)threadIdx.x * NB_PER;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < NB_PER; ++j)
    if (base + j < bytes && tok_start(text, base + j)) ++c;
  // exclusive rank of this thread's starts within the tile
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  __shared__ uint32_t s[BLOCK / WAVE];
  if (lane == 63) s[wave] = inc;
  __syncthreads();
  uint32_t off = toff[blockIdx.x] + inc - c;
  for (int w = 0; w < wave; ++w) off += s[w];
#pragma unroll
  for (int j = 0; j < NB_PER; ++j)
    if (base + j < bytes && tok_start(text, base + j)) tpos[off++] = base + j;
}

// value; flags: 1 = a newline precedes the token (or it is the first), 2 = it opens a
// comment line ('#' or '%' first on its line), 4 = `>>` fails on it, 8 = `>>` reads a
// number from its start but stops inside it (the next `>>` fails there).
// The token as istream >> into an unsigned int reads it (num_get): an optional sign, at
// least one digit, the magnitude at most 2^32 - 1 (else failbit), a '-' wraps modulo 2^32;
// reading stops at the first non-digit.  (4294967295 is a valid value, so validity is a
// flag, not a sentinel.)
__global__ __launch_bounds__(BLOCK) void k_tok_parse(const char *__restrict__ text, uint64_t bytes,
                                                     const uint64_t *__restrict__ tpos, uint64_t ntok,
                                                     uint32_t *__restrict__ val, uint32_t *__restrict__ linestart,
                                                     uint8_t *__restrict__ flags) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; t < ntok; t += stride) {
    const uint64_t p = tpos[t];
    bool nl = p == 0 || t == 0;
    for (uint64_t q = p; q > 0 && blank(text[q - 1]); --q)
      if (text[q - 1] == '\n') { nl = true; break; }
    uint64_t q = p;
    const bool neg = text[q] == '-';
    if (text[q] == '+' || text[q] == '-') ++q;
    uint64_t v = 0;
    int digits = 0;
    for (; q < bytes && text[q] >= '0' && text[q] <= '9'; ++q) {
      v = v * 10 + (uint32_t)(text[q] - '0');
      if (v > 0xFFFFFFFFull) v = 0x100000000ull;   // saturated: overflow stays overflow
      ++digits;
    }
    const bool ok = digits > 0 && v <= 0xFFFFFFFFull;
    const bool rest = ok && q < bytes && !blank(text[q]);
    val[t] = neg ? 0u - (uint32_t)v : (uint32_t)v;
    const char c0 = text[p];
    linestart[t] = nl ? 1u : 0u;
    flags[t] = (nl ? 1 : 0) | (nl && (c0 == '#' || c0 == '%') ? 2 : 0) | (ok ? 0 : 4) | (rest ? 8 : 0);
  }
}

// kept tokens: not on a comment line (skip_comments) ; first bad kept token
__global__ __launch_bounds__(BLOCK) void k_tok_keep(const uint32_t *__restrict__ val, const uint32_t *__restrict__ lineid,
                                                    const uint8_t *__restrict__ flags, const uint8_t *__restrict__ comment,
                                                    uint64_t ntok, int skip_comments, uint32_t *__restrict__ keep,
                                                    unsigned long long *__restrict__ first_bad) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  uint64_t fb = ~0ull;
  for (uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; t < ntok; t += stride) {
    // lineid: inclusive count of line starts up to t, so the token's line is lineid - 1
    const bool dropped = skip_comments && comment[lineid[t] - 1];
    keep[t] = dropped ? 0u : 1u;
    if (!dropped && (flags[t] & 4) && t < fb) fb = t;
    if (!dropped && (flags[t] & 8) && t + 1 < fb) fb = t + 1;   // the input ends right after it
  }
  fb = wave_min(fb);
  if ((threadIdx.x & 63) == 0 && fb != ~0ull) atomicMin(first_bad, (unsigned long long)fb);
}

__global__ void k_line_comment(const uint32_t *__restrict__ lineid, const uint8_t *__restrict__ flags, uint64_t ntok,
                               uint8_t *__restrict__ comment) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; t < ntok; t += stride)
    if (flags[t] & 1) comment[lineid[t] - 1] = (flags[t] & 2) ? 1 : 0;
}

__global__ void k_tok_records(const uint32_t *__restrict__ val, const uint32_t *__restrict__ keep,
                              const uint32_t *__restrict__ kidx, uint64_t limit, uint64_t nrec,
                              sheep_xs1 *__restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; t < limit; t += stride) {
    if (!keep[t]) continue;
    const uint64_t k = kidx[t];
    if (k >= 2 * nrec) continue;
    sheep_xs1 *r = &out[k >> 1];
    if (k & 1) r->head = val[t];
    else { r->tail = val[t]; r->weight = 1.0f; }
  }
}

__global__ void k_add_u32_inplace(uint32_t *__restrict__ dst, const uint32_t *__restrict__ add, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) dst[i] += add[i];
}

// 1 + the largest vid of the records (LLAMA max_nodes) and the self-loop count
__global__ __launch_bounds__(BLOCK) void k_record_stats(const sheep_xs1 *__restrict__ rec, uint64_t nrec,
                                                        unsigned long long *__restrict__ out) {
  uint64_t mx = 0, loops = 0;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nrec; i += stride) {
    const sheep_xs1 r = rec[i];
    const uint64_t v = (uint64_t)(r.tail > r.head ? r.tail : r.head) + 1;
    mx = v > mx ? v : mx;
    loops += r.tail == r.head;
  }
  block_atomic_max(&out[0], mx);
  block_atomic_add(&out[1], loops);
}

}  // namespace

void record_stats(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, uint64_t *max_slot, uint64_t *loops) {
  unsigned long long *d = (unsigned long long *)c.d_scalars + 56;
  HIP_CHECK(hipMemsetAsync(d, 0, 2 * sizeof(uint64_t), c.stream));
  if (nrec) {
    hipLaunchKernelGGL(k_record_stats, dim3(grid_for(nrec)), dim3(BLOCK), 0, c.stream, rec, nrec, d);
    LAUNCH_CHECK();
  }
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 56, d, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  *max_slot = c.h_scalars[56];
  *loops = c.h_scalars[57];
}

uint64_t parse_net(Ctx &c, const char *text, uint64_t bytes, int skip_comments, sheep_xs1 *out, uint64_t cap) {
  if (bytes == 0) return 0;
  const uint64_t ntiles = (bytes + NB_TILE - 1) / NB_TILE;
  uint32_t *tcnt = c.get_as<uint32_t>("net_tcnt", ntiles + 1);
  uint32_t *tot = (uint32_t *)(c.d_scalars + 60);
  hipLaunchKernelGGL(k_tok_count, dim3((unsigned)ntiles), dim3(BLOCK), 0, c.stream, text, bytes, tcnt);
  LAUNCH_CHECK();
  HIP_CHECK(hipMemsetAsync(c.d_scalars + 60, 0, sizeof(uint64_t), c.stream));
  scan_exclusive_u32(c, tcnt, tcnt, ntiles, tot);
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 60, c.d_scalars + 60, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  const uint64_t ntok = (uint32_t)c.h_scalars[60];
  if (ntok == 0) return 0;
  uint64_t *tpos = c.get_as<uint64_t>("net_tpos", ntok);
  hipLaunchKernelGGL(k_tok_write, dim3((unsigned)ntiles), dim3(BLOCK), 0, c.stream, text, bytes, (const uint32_t *)tcnt, tpos);
  LAUNCH_CHECK();
  uint32_t *val = c.get_as<uint32_t>("net_val", ntok), *lineid = c.get_as<uint32_t>("net_lineid", ntok);
  uint8_t *flags = c.get_as<uint8_t>("net_flags", ntok), *comment = c.get_as<uint8_t>("net_comment", ntok);
  hipLaunchKernelGGL(k_tok_parse, dim3(grid_for(ntok)), dim3(BLOCK), 0, c.stream, text, bytes, (const uint64_t *)tpos,
                     ntok, val, lineid, flags);
  LAUNCH_CHECK();
  {   // line starts -> 1-based line id of every token (inclusive scan of the flags)
    uint32_t *ex = c.get_as<uint32_t>("net_lineex", ntok);
    scan_exclusive_u32(c, lineid, ex, ntok, nullptr);
    hipLaunchKernelGGL(k_add_u32_inplace, dim3(grid_for(ntok)), dim3(BLOCK), 0, c.stream, lineid, (const uint32_t *)ex,
                       ntok);
    LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_line_comment, dim3(grid_for(ntok)), dim3(BLOCK), 0, c.stream, (const uint32_t *)lineid,
                     (const uint8_t *)flags, ntok, comment);
  LAUNCH_CHECK();
  uint32_t *keep = c.get_as<uint32_t>("net_keep", ntok + 1), *kidx = c.get_as<uint32_t>("net_kidx", ntok + 1);
  unsigned long long *fb = (unsigned long long *)c.d_scalars + 61;
  HIP_CHECK(hipMemsetAsync(fb, 0xFF, sizeof(uint64_t), c.stream));
  hipLaunchKernelGGL(k_tok_keep, dim3(grid_for(ntok)), dim3(BLOCK), 0, c.stream, (const uint32_t *)val,
                     (const uint32_t *)lineid, (const uint8_t *)flags, (const uint8_t *)comment, ntok, skip_comments,
                     keep, fb);
  LAUNCH_CHECK();
  scan_exclusive_u32(c, keep, kidx, ntok, (uint32_t *)(c.d_scalars + 62));
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 61, c.d_scalars + 61, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  const uint64_t first_bad = c.h_scalars[61];
  const uint64_t limit = first_bad == ~0ull ? ntok : first_bad;
  uint32_t kept = 0;   // kept tokens before the first bad one
  if (limit == ntok) {
    HIP_CHECK(hipMemcpyAsync(&kept, c.d_scalars + 62, sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
  } else {
    HIP_CHECK(hipMemcpyAsync(&kept, kidx + limit, sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
  }
  c.sync();
  const uint64_t nrec = kept / 2;
  if (nrec > cap) throw Error(SHEEP_ERR_ARG, "parse_net: output capacity too small");
  if (nrec)
    hipLaunchKernelGGL(k_tok_records, dim3(grid_for(limit)), dim3(BLOCK), 0, c.stream, (const uint32_t *)val,
                       (const uint32_t *)keep, (const uint32_t *)kidx, limit, nrec, out);
  LAUNCH_CHECK();
  c.sync();
  return nrec;
}

}  // namespace sheep

// ---- .dat partial loads (graph_wrapper.h:43-63: LLAMAGraph(filename, part, num_parts) hands
// lc_partial_load_part / num_parts to the loader, which reads only that part) -------------
// Part p of k is the contiguous record range [(p-1)R/k, pR/k) of the R = size / 12 records;
// the host reads exactly those bytes with pread, never the rest of the file.
extern "C" int sheep_dat_range(const char *filename, uint64_t part, uint64_t num_parts, uint64_t *first_out,
                               uint64_t *count_out) {
  try {
    if (!filename || !first_out || !count_out) throw sheep::Error(SHEEP_ERR_ARG, "null argument");
    if (num_parts != 0 && (part < 1 || part > num_parts)) throw sheep::Error(SHEEP_ERR_ARG, "part must be in 1..num_parts");
    struct stat st;
    if (stat(filename, &st) != 0) throw sheep::Error(SHEEP_ERR_ARG, std::string("cannot open ") + filename);
    const uint64_t R = (uint64_t)st.st_size / sizeof(sheep_xs1);
    uint64_t beg = 0, end = R;
    if (num_parts != 0) {
      beg = (part - 1) * R / num_parts;   // (R < 2^40: no overflow for any part count < 2^24)
      end = part * R / num_parts;
    }
    *first_out = beg;
    *count_out = end - beg;
    return SHEEP_OK;
  } catch (const sheep::Error &e) {
    sheep::set_error(e.what());
    return e.code;
  }
}

extern "C" int sheep_read_dat(const char *filename, uint64_t first, uint64_t count, sheep_xs1 *out, uint64_t *got_out) {
  int fd = -1;
  try {
    if (!filename || !got_out || (count && !out)) throw sheep::Error(SHEEP_ERR_ARG, "null argument");
    *got_out = 0;
    fd = open(filename, O_RDONLY);
    if (fd < 0) throw sheep::Error(SHEEP_ERR_ARG, std::string("cannot open ") + filename);
    char *dst = (char *)out;
    uint64_t left = count * sizeof(sheep_xs1), off = first * sizeof(sheep_xs1);
    while (left) {
      const ssize_t r = pread(fd, dst, left > (1ull << 30) ? (1ull << 30) : left, (off_t)off);
      if (r < 0 && errno == EINTR) continue;
      if (r < 0) throw sheep::Error(SHEEP_ERR_ARG, std::string("read ") + filename + ": " + strerror(errno));
      if (r == 0) break;   // (the file shrank)
      dst += r;
      off += (uint64_t)r;
      left -= (uint64_t)r;
    }
    close(fd);
    *got_out = (count * sizeof(sheep_xs1) - left) / sizeof(sheep_xs1);
    return SHEEP_OK;
  } catch (const sheep::Error &e) {
    if (fd >= 0) close(fd);
    sheep::set_error(e.what());
    return e.code;
  }
}
