// Offpolicy episode replay on the device: RecReplayBuffer / PrioritizedRecReplayBuffer
// (offpolicy/utils/rec_buffer.py:10-324) and SumSegmentTree / MinSegmentTree
// (offpolicy/utils/segment_tree.py:18-165).
//
// Episodes are whole-sequence records; a field's store is [slot][L][row] so one episode of one
// field is a contiguous run and an insert / gather is pure HBM byte movement: one launch moves
// every field (blockIdx.y = field), thread per float, consecutive threads on consecutive floats of
// a row on both sides. The trees are f64 heaps (root 1, leaves itcap + i, the reference layout);
// their ops touch a handful of nodes per call, so each is ONE single-workgroup launch: leaf writes,
// then the written leaves' ancestors re-derived level by level as op(left, right) — identical values
// to the reference's unique()-per-level loop whatever the order, since every node is a pure
// function of its two children.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "common.h"
#include "minimarl.h"

struct mm_erb {
  mm_erb_dims d;
  int64_t size, itcap, filled, current;
  float alpha_f;     // numpy: float32 priorities ** Python-float alpha -> the alpha is cast to float32
  void* alloc;
  float* f[6];       // obs, share, acts, rew, dones, dones_env stores [size][L][R]
  int L[6];
  int R[6];
  double* sum;
  double* mn;
  float* maxp;
  int32_t* err;
};

namespace mm {

struct ErbField {
  float* store;
  const float* src;    // insert source (reference insert layout) / unused in gather
  float* dst;          // gather destination (sample layout) / unused in insert
  uint32_t L, R;       // steps, floats per (slot, step) in the store
  uint32_t R_in;       // insert: floats per (step, episode) in the source (>= R: share keeps agent 0)
  uint32_t Nf;         // gather: agent split of a row (row = Nf x X) -> [Nf, L, B, X]
};
struct ErbFieldSet {
  ErbField f[6];
  int nf;
};

// insert: store[(slot(e) L + l) R + r] = src[(l n + e) R_in + r], slot(e) = (current + e) % size
__global__ __launch_bounds__(256) void erb_insert_kernel(ErbFieldSet fs, uint32_t n, int64_t current, int64_t size) {
  const ErbField& F = fs.f[blockIdx.y];
  const uint64_t total = (uint64_t)F.L * n * F.R;
  for (uint64_t o = (uint64_t)blockIdx.x * 256 + threadIdx.x; o < total; o += (uint64_t)gridDim.x * 256) {
    const uint64_t r = o % F.R, le = o / F.R, e = le % n, l = le / n;
    const int64_t slot = (current + e) % size;
    F.store[((size_t)slot * F.L + l) * F.R + r] = F.src[((size_t)l * n + e) * F.R_in + r];
  }
}

// gather (sample_inds): dst[((nf L + l) B + b) X + x] = store[(idx_b L + l) R + nf X + x]
// (an index outside [0, size) reads nothing: its rows are written as 0 and bit 2 of err is set)
__global__ __launch_bounds__(256) void erb_gather_kernel(ErbFieldSet fs, uint32_t B, const int64_t* __restrict__ idx,
                                                         int64_t size, int32_t* err) {
  const ErbField& F = fs.f[blockIdx.y];
  const uint32_t X = F.R / F.Nf;
  const uint64_t total = (uint64_t)F.L * B * F.R;
  for (uint64_t o = (uint64_t)blockIdx.x * 256 + threadIdx.x; o < total; o += (uint64_t)gridDim.x * 256) {
    const uint64_t x = o % X, q = o / X, b = q % B, q2 = q / B, l = q2 % F.L, nf = q2 / F.L;
    const int64_t slot = idx[b];
    if (slot < 0 || slot >= size) {
      F.dst[o] = 0.0f;
      if (o == 0 || x + l + nf == 0) atomicOr(err, 4);
      continue;
    }
    F.dst[o] = F.store[((size_t)slot * F.L + l) * F.R + nf * X + x];
  }
}

// f32 pow as numpy computes float32 ** float32 (correctly rounded via an f64 pow)
__device__ __forceinline__ double prio_pow(float p, float a) { return (double)(float)pow((double)p, (double)a); }

// Leaf writes + ancestor re-derivation for n entries. Entry i: leaf idx_i = idx ? idx[i] : (base + i) % mod,
// value = prio ? prio[i] ** a : maxp ** a. Duplicates: the last entry wins (numpy fancy assignment).
// check_len >= 0: entries with idx outside [0, check_len) or prio <= 0 are skipped and flagged in err.
__global__ __launch_bounds__(1024) void erb_set_kernel(double* __restrict__ sum, double* __restrict__ mn, int64_t itcap,
                                                       int n, const int64_t* __restrict__ idx, int64_t base,
                                                       int64_t mod, const float* __restrict__ prio, float* maxp,
                                                       float a, int64_t check_len, int32_t* err) {
  __shared__ float red[1024];
  __shared__ int depth_s;
  const int tid = threadIdx.x;
  const float mp = *maxp;
  float local_max = 0.f;
  int bad = 0;
  for (int i = tid; i < n; i += 1024) {
    const int64_t k = idx ? idx[i] : (base + i) % mod;
    bool ok = k >= 0 && k < itcap;
    if (check_len >= 0 && !(k >= 0 && k < check_len)) { ok = false; bad |= 1; }
    float p = mp;
    if (prio) {
      p = prio[i];
      if (!(p > 0.f)) { ok = false; bad |= 2; }
      local_max = fmaxf(local_max, p);
    }
    if (!ok) continue;
    bool later = false;
    if (idx)
      for (int j = i + 1; j < n && !later; ++j) later = idx[j] == k;
    if (later) continue;
    const double v = prio_pow(p, a);
    sum[itcap + k] = v;
    mn[itcap + k] = v;
  }
  if (bad && err) atomicOr(err, bad);
  red[tid] = local_max;
  if (tid == 0) depth_s = 63 - __clzll((unsigned long long)itcap);
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if (tid < s) red[tid] = fmaxf(red[tid], red[tid + s]);
    __syncthreads();
  }
  // ancestors, one tree level per barrier (children final before parents read them)
  const int depth = depth_s;
  for (int lv = 1; lv <= depth; ++lv) {
    for (int i = tid; i < n; i += 1024) {
      const int64_t k = idx ? idx[i] : (base + i) % mod;
      if (k < 0 || k >= itcap) continue;
      const int64_t p = (itcap + k) >> lv;
      const double l0 = sum[2 * p], r0 = sum[2 * p + 1];
      sum[p] = l0 + r0;
      const double l1 = mn[2 * p], r1 = mn[2 * p + 1];
      mn[p] = l1 < r1 ? l1 : r1;
    }
    __syncthreads();
  }
  if (prio && tid == 0 && red[0] > mp) *maxp = red[0];   // max(max_priorities, np.max(priorities))
}

__device__ __forceinline__ double rng_unit53(uint64_t r) { return (double)(r >> 11) * (1.0 / 9007199254740992.0); }

// Prioritized sample: total = _it_sums.sum(0, len - 1) (rec_buffer.py:273). SegmentTree.reduce
// decrements its end (segment_tree.py:71), so the fold covers leaves [0, len - 2] — the last filled
// leaf is never part of the sampled mass. Folded in the reference's _reduce_helper order (start 0: a
// right fold of the fully covered left children met on the way down to the node whose range ends at
// len - 2), then per draw the prefix-sum descent and the IS weight.
__global__ __launch_bounds__(256) void erb_sample_kernel(const double* __restrict__ sum, const double* __restrict__ mn,
                                                         int64_t itcap, int64_t len, int B, double beta,
                                                         const double* __restrict__ fracs, uint64_t seed,
                                                         uint64_t counter, int64_t* __restrict__ idx_out,
                                                         double* __restrict__ w_out, float* __restrict__ w32_out) {
  __shared__ double total_s;
  if (threadIdx.x == 0) {
    int64_t node = 1, ns = 0, ne = itcap - 1;
    const int64_t end = len - 2;   // len > B >= 1 (checked on the host)
    int64_t lefts[64];
    int nl = 0;
    while (end != ne) {
      const int64_t mid = (ns + ne) >> 1;
      if (end <= mid) {
        node = 2 * node;
        ne = mid;
      } else {
        lefts[nl++] = 2 * node;
        node = 2 * node + 1;
        ns = mid + 1;
      }
    }
    double acc = sum[node];
    while (nl > 0) acc = sum[lefts[--nl]] + acc;
    total_s = acc;
  }
  __syncthreads();
  const double total = total_s, root = sum[1];
  const double max_w = pow(mn[1] / root * (double)len, -beta);
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const double u = fracs ? fracs[b] : rng_unit53(rng_draw(seed, counter, (uint64_t)b, 0x5E6ull));
    double mass = u * total;
    int64_t k = 1;
    while (k < itcap) {
      k *= 2;
      const double v = sum[k];
      if (v <= mass) {
        mass -= v;
        k += 1;
      }
    }
    const int64_t leaf = k - itcap;
    idx_out[b] = leaf;
    const double w = pow(sum[k] / root * (double)len, -beta) / max_w;
    if (w_out) w_out[b] = w;
    if (w32_out) w32_out[b] = (float)w;
  }
}

__global__ __launch_bounds__(256) void erb_uniform_kernel(int64_t len, int B, uint64_t seed, uint64_t counter,
                                                          int64_t* __restrict__ idx_out) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  int64_t k = (int64_t)(rng_unit53(rng_draw(seed, counter, (uint64_t)b, 0x0E1ull)) * (double)len);
  idx_out[b] = k < len ? k : len - 1;
}

}  // namespace mm

namespace {
const int kFieldRows = 6;

int erb_grid(const mm::ErbFieldSet& fs, uint32_t units) {
  uint64_t mx = 0;
  for (int i = 0; i < fs.nf; ++i) mx = std::max<uint64_t>(mx, (uint64_t)fs.f[i].L * units * fs.f[i].R);
  uint64_t g = (mx + 255) / 256;
  return (int)std::min<uint64_t>(std::max<uint64_t>(g, 1), 2048);
}
}  // namespace

extern "C" {

int mm_erb_create(const mm_erb_dims* d, int64_t buffer_size, double alpha, mm_erb** out) {
  MM_REQUIRE(d && out && buffer_size >= 1 && buffer_size < (1ll << 30), "erb_create: bad arguments");
  MM_REQUIRE(d->T >= 1 && d->N >= 1 && d->D >= 1 && d->S >= 1 && d->A >= 1, "erb_create: bad dims");
  mm_erb* b = new mm_erb;
  b->d = *d;
  b->size = buffer_size;
  b->itcap = 1;
  while (b->itcap < buffer_size) b->itcap *= 2;
  b->filled = b->current = 0;
  b->alpha_f = (float)alpha;
  const int T = d->T, N = d->N;
  const int L[kFieldRows] = {T + 1, T + 1, T, T, T, T};
  const int R[kFieldRows] = {N * d->D, d->same_share ? d->S : N * d->S, N * d->A, N, N, 1};
  size_t off[kFieldRows + 1];
  off[0] = 0;
  for (int i = 0; i < kFieldRows; ++i) {
    b->L[i] = L[i];
    b->R[i] = R[i];
    MM_REQUIRE((uint64_t)L[i] * R[i] * (uint64_t)std::max<int64_t>(buffer_size, 1) < (1ull << 40), "erb_create: too large");
    off[i + 1] = off[i] + (((size_t)buffer_size * L[i] * R[i] * 4 + 255) & ~size_t(255));
  }
  const size_t tree_b = ((size_t)2 * b->itcap * 8 + 255) & ~size_t(255);
  const size_t total = off[kFieldRows] + 2 * tree_b + 256;
  void* base = nullptr;
  if (hipMalloc(&base, total) != hipSuccess) {
    delete b;
    mm::set_error("erb_create: hipMalloc of %zu bytes failed", total);
    return MM_ENOMEM;
  }
  b->alloc = base;
  char* p = static_cast<char*>(base);
  for (int i = 0; i < kFieldRows; ++i) b->f[i] = reinterpret_cast<float*>(p + off[i]);
  b->sum = reinterpret_cast<double*>(p + off[kFieldRows]);
  b->mn = reinterpret_cast<double*>(p + off[kFieldRows] + tree_b);
  b->maxp = reinterpret_cast<float*>(p + off[kFieldRows] + 2 * tree_b);
  b->err = reinterpret_cast<int32_t*>(p + off[kFieldRows] + 2 * tree_b + 4);
  // stores zero, dones / dones_env one (rec_buffer.py:120-141: "default to done being True")
  std::vector<double> inf_tree(2 * b->itcap, INFINITY);
  const float one = 1.0f;
  bool ok = hipMemset(base, 0, off[kFieldRows] + tree_b) == hipSuccess &&
            hipMemcpy(b->mn, inf_tree.data(), 2 * b->itcap * 8, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(b->maxp, &one, 4, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemset(b->err, 0, 4) == hipSuccess;
  for (int i = 4; i < kFieldRows && ok; ++i) {
    const size_t n = (size_t)buffer_size * L[i] * R[i];
    ok = hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(b->f[i]), 0x3f800000, n) == hipSuccess;
  }
  if (!ok || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(base);
    delete b;
    mm::set_error("erb_create: init failed");
    return MM_EHIP;
  }
  *out = b;
  return MM_OK;
}

void mm_erb_destroy(mm_erb* b) {
  if (!b) return;
  (void)hipFree(b->alloc);
  delete b;
}

int mm_erb_insert(mm_erb* b, int32_t n, const mm_erb_fields* src, int64_t* idx_range_host, mm_stream_t s) {
  MM_REQUIRE(b && src && n >= 1 && n <= b->size, "erb_insert: bad arguments (n must be in [1, buffer_size])");
  const float* in[kFieldRows] = {src->obs, src->share_obs, src->acts, src->rewards, src->dones, src->dones_env};
  mm::ErbFieldSet fs;
  fs.nf = kFieldRows;
  for (int i = 0; i < kFieldRows; ++i) {
    MM_REQUIRE(in[i] != nullptr, "erb_insert: field %d is NULL", i);
    fs.f[i] = {b->f[i], in[i], nullptr, (uint32_t)b->L[i], (uint32_t)b->R[i], (uint32_t)b->R[i], 1u};
  }
  if (b->d.same_share) fs.f[1].R_in = (uint32_t)(b->d.N * b->d.S);   // [T+1, n, N, S] -> agent 0
  hipStream_t st = (hipStream_t)s;
  hipLaunchKernelGGL(mm::erb_insert_kernel, dim3(erb_grid(fs, n), kFieldRows), dim3(256), 0, st, fs, (uint32_t)n,
                     b->current, b->size);
  MM_HIP_CHECK(hipGetLastError());
  const int64_t first = b->current;
  if (b->d.prioritized) {
    // reference: leaves 0..n-1 (range(len(idx_range))); slots mode: the ring slots just written
    const int64_t base = b->d.leaf_mode ? first : 0, mod = b->d.leaf_mode ? b->size : (int64_t)n;
    hipLaunchKernelGGL(mm::erb_set_kernel, dim3(1), dim3(1024), 0, st, b->sum, b->mn, b->itcap, (int)n,
                       (const int64_t*)nullptr, base, mod, (const float*)nullptr, b->maxp, b->alpha_f, (int64_t)-1,
                       (int32_t*)nullptr);
    MM_HIP_CHECK(hipGetLastError());
  }
  if (idx_range_host)
    for (int i = 0; i < n; ++i) idx_range_host[i] = (first + i) % b->size;
  b->current = (first + n - 1) % b->size + 1;
  b->filled = std::min<int64_t>(b->filled + n, b->size);
  return MM_OK;
}

int64_t mm_erb_len(const mm_erb* b) { return b ? b->filled : -1; }
int64_t mm_erb_current(const mm_erb* b) { return b ? b->current : -1; }
int64_t mm_erb_it_capacity(const mm_erb* b) { return b ? b->itcap : -1; }

int mm_erb_sample_prioritized(mm_erb* b, int32_t B, double beta, const double* fracs, uint64_t seed,
                              uint64_t counter, int64_t* idx_out, double* w_out, float* w32_out, mm_stream_t s) {
  MM_REQUIRE(b && b->d.prioritized && idx_out && B >= 1, "erb_sample_prioritized: bad arguments");
  MM_REQUIRE(b->filled > B, "erb_sample_prioritized: Cannot sample with no completed episodes in the buffer! "
                            "(len %lld <= batch %d)", (long long)b->filled, B);
  MM_REQUIRE(beta > 0, "erb_sample_prioritized: beta must be > 0");
  hipLaunchKernelGGL(mm::erb_sample_kernel, dim3(1), dim3(256), 0, (hipStream_t)s, b->sum, b->mn, b->itcap,
                     b->filled, (int)B, beta, fracs, seed, counter, idx_out, w_out, w32_out);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_erb_sample_uniform(mm_erb* b, int32_t B, uint64_t seed, uint64_t counter, int64_t* idx_out, mm_stream_t s) {
  MM_REQUIRE(b && idx_out && B >= 1 && b->filled >= 1, "erb_sample_uniform: bad arguments / empty buffer");
  hipLaunchKernelGGL(mm::erb_uniform_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)s, b->filled, (int)B,
                     seed, counter, idx_out);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_erb_gather(mm_erb* b, int32_t B, const int64_t* idx, const mm_erb_fields* dst, mm_stream_t s) {
  MM_REQUIRE(b && idx && dst && B >= 1, "erb_gather: bad arguments");
  float* out[kFieldRows] = {dst->obs, dst->share_obs, dst->acts, dst->rewards, dst->dones, dst->dones_env};
  const uint32_t split[kFieldRows] = {(uint32_t)b->d.N, b->d.same_share ? 1u : (uint32_t)b->d.N, (uint32_t)b->d.N,
                                      (uint32_t)b->d.N, (uint32_t)b->d.N, 1u};
  mm::ErbFieldSet fs;
  fs.nf = 0;
  for (int i = 0; i < kFieldRows; ++i) {
    if (!out[i]) continue;
    fs.f[fs.nf++] = {b->f[i], nullptr, out[i], (uint32_t)b->L[i], (uint32_t)b->R[i], (uint32_t)b->R[i], split[i]};
  }
  if (fs.nf == 0) return MM_OK;
  hipLaunchKernelGGL(mm::erb_gather_kernel, dim3(erb_grid(fs, B), fs.nf), dim3(256), 0, (hipStream_t)s, fs, (uint32_t)B,
                     idx, b->size, b->err);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_erb_update_priorities(mm_erb* b, const int64_t* idx, const float* prio, int32_t B, mm_stream_t s) {
  MM_REQUIRE(b && b->d.prioritized && idx && prio && B >= 1, "erb_update_priorities: bad arguments");
  hipLaunchKernelGGL(mm::erb_set_kernel, dim3(1), dim3(1024), 0, (hipStream_t)s, b->sum, b->mn, b->itcap, (int)B, idx,
                     (int64_t)0, (int64_t)1, prio, b->maxp, b->alpha_f, b->filled, b->err);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

double* mm_erb_sum_tree(mm_erb* b) { return b ? b->sum : nullptr; }
double* mm_erb_min_tree(mm_erb* b) { return b ? b->mn : nullptr; }
float* mm_erb_max_priority(mm_erb* b) { return b ? b->maxp : nullptr; }
int32_t* mm_erb_error_word(mm_erb* b) { return b ? b->err : nullptr; }

int mm_erb_copy_state(mm_erb* b, double* sum_dst, double* min_dst, float* maxp_dst, int32_t* err_dst, mm_stream_t s) {
  MM_REQUIRE(b, "erb_copy_state: NULL handle");
  hipStream_t st = (hipStream_t)s;
  const size_t tb = (size_t)2 * b->itcap * 8;
  if (sum_dst) MM_HIP_CHECK(hipMemcpyAsync(sum_dst, b->sum, tb, hipMemcpyDeviceToDevice, st));
  if (min_dst) MM_HIP_CHECK(hipMemcpyAsync(min_dst, b->mn, tb, hipMemcpyDeviceToDevice, st));
  if (maxp_dst) MM_HIP_CHECK(hipMemcpyAsync(maxp_dst, b->maxp, 4, hipMemcpyDeviceToDevice, st));
  if (err_dst) MM_HIP_CHECK(hipMemcpyAsync(err_dst, b->err, 4, hipMemcpyDeviceToDevice, st));
  return MM_OK;
}

}  // extern "C"
