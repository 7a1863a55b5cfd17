// dlagg.hip — the accdfl FedAvg weighted N-peer reduce for MI355X (gfx950, CDNA4).
//
// Replaces the torch-CPU loop of accdfl/core/gradient_aggregation/fedavg.py:20-25:
//     center = deepcopy(models[0]); p.mul_(0)           (:20-22)
//     for m, w in zip(models, weights):                  (:23)
//         for c1, p1 in zip(center.parameters(), m.parameters()):  (:24)
//             c1.add_(w * p1)                            (:25)
// as ONE streaming pass over HBM: every peer byte is read once, every output byte
// written once, the running sum lives in VGPRs.  Per element the peers are folded
// in list order with separately rounded multiply and add (no FMA), which is the
// reference's rounding sequence bit for bit (see include/dlagg.h).
//
// Roofline: 2 flop per 4..8 B read -> far below the MFMA ridge; the kernel is
// HBM-bound and deliberately has no MFMA.  Algorithmic bytes per launch =
// (n_peers + 1) * n_elems * sizeof(T).
//
// Layout of the work: one 16-byte chunk per lane per peer (global_load_dwordx4,
// 1 KiB per wave instruction, fully coalesced), CH chunks per lane per tile,
// peers loaded in groups of 8 so each lane keeps 8*CH*16 B in flight before the
// first add.  Loads are non-temporal (each byte is read once); the output is
// stored sc1 (write-through, not kept in the XCD L2), which measured +3.5 % over
// plain stores on the 8 x 25 M fp32 north-star reduce (profiles/r01_*).  No LDS in
// the stream: each lane folds only its own elements, so there is no cross-lane
// exchange to stage, and LDS-DMA staging buys nothing for a pure stream at this
// occupancy (the register stream already keeps >300 KiB in flight per CU).  LDS is
// used only to transpose the peers' values of a ragged tail (< one chunk), which
// one wave gathers lane-parallel in its own workgroup.
// Small shares over many peers take a word-per-lane kernel (wsum_wide_kernel) that
// keeps up to 64 peers' loads in flight per lane.
//
// Compiled with -ffp-contract=off; the pragma below repeats it so no build line
// can re-enable FMA contraction for these functions.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <new>
#include <set>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include <unistd.h>

#include "dlagg.h"

// Hash of this file, include/dlagg.h and the compile flags, set by the build
// (accdfl_amd/_lib.py build()); the loader refuses a library whose id differs from the tree's.
#ifndef DLA_BUILD_ID
#define DLA_BUILD_ID "unversioned"
#endif

namespace {

// Embedded as plain bytes too, so a build's id can be read from the file without loading it.
__attribute__((used)) const char kBuildIdTag[] = "dlagg-build-id:" DLA_BUILD_ID;

constexpr int kBlock = 256;           // multi-tensor / scalar kernels: 4 waves of 64 lanes
constexpr int kGroup = 8;             // peers loaded together before folding
constexpr int kMaxPeersPerPass = 128; // pointer table in the kernel-argument block

thread_local std::string g_last_error;

// A/B knobs (environment variables such as DLA_VEC_WGS_PER_CU) exist only in the tuning build
// (-DDLA_TUNING=1 -> lib/libdlagg_tuning.so, loaded when ACCDFL_AMD_TUNING=1; profiles/ scripts
// use it); the product library reads no environment and runs the measured policy.
#ifndef DLA_TUNING
#define DLA_TUNING 0
#endif
inline const char* tuning_env(const char* name) {
  return DLA_TUNING ? std::getenv(name) : nullptr;
}

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

// ---------------------------------------------------------------- element ops
// One 16-byte chunk = E elements.  acc_t is the op-math type; values of acc are
// always exactly representable in the storage dtype (the reference stores the
// running sum in the parameter tensor after every add).

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int DT> struct Ops;

template <> struct Ops<DLA_F32> {
  using acc_t = float;
  using w_t = float;
  using elem_t = float;
  static constexpr int E = 4;
  __device__ static void unpack(const uint4& v, acc_t* x) {
    x[0] = __uint_as_float(v.x); x[1] = __uint_as_float(v.y);
    x[2] = __uint_as_float(v.z); x[3] = __uint_as_float(v.w);
  }
  __device__ static uint4 pack(const acc_t* a) {
    return make_uint4(__float_as_uint(a[0]), __float_as_uint(a[1]),
                      __float_as_uint(a[2]), __float_as_uint(a[3]));
  }
  __device__ static acc_t to_acc(elem_t e) { return e; }
  __device__ static elem_t from_acc(acc_t a) { return a; }
  __device__ static acc_t zero_mul(acc_t x) { return x * 0.0f; }                 // fedavg.py:22
  __device__ static acc_t step(acc_t acc, w_t w, acc_t x) { return acc + w * x; } // fedavg.py:25
  // one word per lane in the wide kernel: 4 bytes = 1 element
  using word_t = uint32_t;
  static constexpr int WE = 1;
  __device__ static void unpack_w(word_t v, acc_t* x) { x[0] = __uint_as_float(v); }
  __device__ static word_t pack_w(const acc_t* a) { return __float_as_uint(a[0]); }
};

template <> struct Ops<DLA_F64> {
  using acc_t = double;
  using w_t = double;
  using elem_t = double;
  static constexpr int E = 2;
  __device__ static void unpack(const uint4& v, acc_t* x) {
    x[0] = __hiloint2double(v.y, v.x);
    x[1] = __hiloint2double(v.w, v.z);
  }
  __device__ static uint4 pack(const acc_t* a) {
    return make_uint4(__double2loint(a[0]), __double2hiint(a[0]),
                      __double2loint(a[1]), __double2hiint(a[1]));
  }
  __device__ static acc_t to_acc(elem_t e) { return e; }
  __device__ static elem_t from_acc(acc_t a) { return a; }
  __device__ static acc_t zero_mul(acc_t x) { return x * 0.0; }
  __device__ static acc_t step(acc_t acc, w_t w, acc_t x) { return acc + w * x; }
  using word_t = u32x2;  // 8 bytes = 1 element
  static constexpr int WE = 1;
  __device__ static void unpack_w(word_t v, acc_t* x) { x[0] = __hiloint2double(v.y, v.x); }
  __device__ static word_t pack_w(const acc_t* a) {
    word_t w = {static_cast<uint32_t>(__double2loint(a[0])), static_cast<uint32_t>(__double2hiint(a[0]))};
    return w;
  }
};

// bf16: op-math float, every product and every sum rounded RNE to bf16
// (torch-CPU reduced-float kernels: float(a) * float(w) -> bf16; float(c) + float(t) -> bf16).
__device__ inline float bf16_bits_to_f(uint32_t h) { return __uint_as_float(h << 16); }
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ inline float round_bf16(float f) {
  // v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN stays NaN) with a zero LOW operand: the rounded
  // bf16 lands in the high half over a zero low half, which IS the rounded value's f32 bit pattern
  // — one instruction, where a cast back to f32 costs a cvt plus a shift or mask per element.
  const bf16x2 h = __builtin_convertvector(f32x2{0.0f, f}, bf16x2);
  uint32_t bits;
  __builtin_memcpy(&bits, &h, 4);
  return __uint_as_float(bits);
}

template <> struct Ops<DLA_BF16> {
  using acc_t = float;
  using w_t = float;
  using elem_t = uint16_t;
  static constexpr int E = 8;
  __device__ static void unpack(const uint4& v, acc_t* x) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[2 * i] = __uint_as_float(w[i] << 16);
      x[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  // acc values are exact bf16 values: their upper 16 bits are the bf16 bits.
  __device__ static uint4 pack(const acc_t* a) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = (__float_as_uint(a[2 * i]) >> 16) | (__float_as_uint(a[2 * i + 1]) & 0xffff0000u);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
  __device__ static acc_t to_acc(elem_t e) { return bf16_bits_to_f(e); }
  __device__ static elem_t from_acc(acc_t a) { return static_cast<uint16_t>(__float_as_uint(a) >> 16); }
  __device__ static acc_t zero_mul(acc_t x) { return x * 0.0f; }  // +-0 or NaN: already bf16-exact
  __device__ static acc_t step(acc_t acc, w_t w, acc_t x) {
    return round_bf16(acc + round_bf16(w * x));
  }
  using word_t = uint32_t;  // 4 bytes = 2 elements
  static constexpr int WE = 2;
  __device__ static void unpack_w(word_t v, acc_t* x) {
    x[0] = __uint_as_float(v << 16);
    x[1] = __uint_as_float(v & 0xffff0000u);
  }
  __device__ static word_t pack_w(const acc_t* a) {
    return (__float_as_uint(a[0]) >> 16) | (__float_as_uint(a[1]) & 0xffff0000u);
  }
};

// Two bf16 FedAvg steps on one 32-bit word of two bf16 values (element 0 in the low half):
// acc[e] = R(acc[e] + R(w * x[e])), R = RNE to bf16, op-math fp32 — Ops<DLA_BF16>::step on
// both elements, with packed fp32 ops and one conversion per element per rounding
// (round_bf16: 8 VALU per word and step against 10 for one packed conversion + shift + mask).
__device__ inline f32x2 round_bf16x2(f32x2 v) { return f32x2{round_bf16(v.x), round_bf16(v.y)}; }
__device__ inline void bf16_step2(float& a0, float& a1, float w, uint32_t word) {
  const f32x2 x = {__uint_as_float(word << 16), __uint_as_float(word & 0xffff0000u)};
  const f32x2 prod = round_bf16x2(x * w);               // fedavg.py:25 w * p1
  const f32x2 sum = round_bf16x2(f32x2{a0, a1} + prod);  // c1.add_(...)
  a0 = sum.x;
  a1 = sum.y;
}
__device__ inline void bf16_step2(float (&acc)[2], float w, uint32_t word) { bf16_step2(acc[0], acc[1], w, word); }

__device__ inline float half_bits_to_f(uint32_t h) {
  _Float16 v;
  uint16_t s = static_cast<uint16_t>(h);
  __builtin_memcpy(&v, &s, 2);
  return static_cast<float>(v);
}
__device__ inline uint32_t f_to_half_bits(float f) {
  _Float16 v = static_cast<_Float16>(f);  // RNE
  uint16_t s;
  __builtin_memcpy(&s, &v, 2);
  return s;
}
// The empty asm pins the op-math product/sum as a rounded f32 in a VGPR before the
// f16 rounding: without it the backend folds fptrunc(fmul) into one
// v_fma_mixlo_f16 (a single rounding), which differs from the reference's
// f32-then-f16 double rounding on rare ties.
__device__ inline float pin(float f) {
  asm("" : "+v"(f));
  return f;
}
__device__ inline float round_f16(float f) { return static_cast<float>(static_cast<_Float16>(pin(f))); }

// Two f16 FedAvg steps on one 32-bit word of two f16 values (element 0 in the low half), as
// Ops<DLA_F16>::step on both: packed fp32 multiply / add, one v_cvt_pk_f16_f32 (RNE) per
// rounding.  The product and the sum are pinned as rounded fp32 pairs first, for the same
// reason as pin(): no fused mix-precision form may skip the fp32 rounding.
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
__device__ inline f32x2 pin2(f32x2 v) {
  asm("" : "+v"(v));
  return v;
}
__device__ inline f32x2 round_f16x2(f32x2 v) {
  const f16x2 h = __builtin_convertvector(pin2(v), f16x2);  // v_cvt_pk_f16_f32
  return __builtin_convertvector(h, f32x2);
}
__device__ inline void f16_step2(float& a0, float& a1, float w, uint32_t word) {
  f16x2 xh;
  __builtin_memcpy(&xh, &word, 4);
  const f32x2 x = __builtin_convertvector(xh, f32x2);
  const f32x2 prod = round_f16x2(x * w);               // fedavg.py:25 w * p1
  const f32x2 sum = round_f16x2(f32x2{a0, a1} + prod);  // c1.add_(...)
  a0 = sum.x;
  a1 = sum.y;
}

template <> struct Ops<DLA_F16> {
  using acc_t = float;
  using w_t = float;
  using elem_t = uint16_t;
  static constexpr int E = 8;
  __device__ static void unpack(const uint4& v, acc_t* x) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[2 * i] = half_bits_to_f(w[i] & 0xffffu);
      x[2 * i + 1] = half_bits_to_f(w[i] >> 16);
    }
  }
  __device__ static uint4 pack(const acc_t* a) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = f_to_half_bits(a[2 * i]) | (f_to_half_bits(a[2 * i + 1]) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
  __device__ static acc_t to_acc(elem_t e) { return half_bits_to_f(e); }
  __device__ static elem_t from_acc(acc_t a) { return static_cast<uint16_t>(f_to_half_bits(a)); }
  __device__ static acc_t zero_mul(acc_t x) { return x * 0.0f; }  // +-0 or NaN: already f16-exact
  __device__ static acc_t step(acc_t acc, w_t w, acc_t x) { return round_f16(acc + round_f16(w * x)); }
  using word_t = uint32_t;  // 4 bytes = 2 elements
  static constexpr int WE = 2;
  __device__ static void unpack_w(word_t v, acc_t* x) {
    x[0] = half_bits_to_f(v & 0xffffu);
    x[1] = half_bits_to_f(v >> 16);
  }
  __device__ static word_t pack_w(const acc_t* a) { return f_to_half_bits(a[0]) | (f_to_half_bits(a[1]) << 16); }
};

// ------------------------------------------------------------ kernel arguments

template <typename W, int KMAX>
struct PeerTable {
  const void* p[KMAX];
  W w[KMAX];
};

template <bool NT>
__device__ inline uint4 load16(const uint4* p) {
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
  u32x4 v;
  if constexpr (NT) {
    v = __builtin_nontemporal_load(q);  // global_load_dwordx4 ... nt
  } else {
    v = *q;
  }
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Store policy: 0 plain, 1 nt, 2 sc1 (drops the line from the XCD L2), 3 sc0 sc1.
template <int SP>
__device__ inline void store16(uint4* p, const uint4& v) {
  u32x4 w = {v.x, v.y, v.z, v.w};
  if constexpr (SP == 1) {
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));  // global_store_dwordx4 ... nt
  } else if constexpr (SP == 2) {
    // s_nop 1 inside the string: a store of more than 8 bytes reads its data VGPRs after
    // issue, and hipcc does not pad an asm store, so its next VALU could overwrite them.
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
  } else if constexpr (SP == 3) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
  } else {
    *reinterpret_cast<u32x4*>(p) = w;
  }
}

// ------------------------------------------------------------ tile bodies
//
// fold_tile: one tile = BS * CH chunks; lane l of the block owns chunks
// base0 + c*BS + l.  Peers are folded in list order, loaded in groups of
// kGroup so a group's kGroup*CH loads all issue before the first wait.
// ACC_IN: the running sum starts from `out` (second and later passes of a reduce
// with more than KMAX peers) instead of p0 * 0.
// One peer's 16-byte chunk folded into its E running sums (fedavg.py:22 when `first`, then
// fedavg.py:25).  PK: 16-bit pairs through bf16_step2 / f16_step2 (packed fp32 ops, one
// packed conversion per rounding).  fold_tile uses it for peer tables of more than 8
// (16 x 21.3 M bf16 121.9 -> 118.8 us, f16 168.3 -> 118.9) and for f16 groups of 8 with
// smaller tables (8 x 50 M f16 191.8 -> 142.4).  bf16 tables of <= 8 peers and the
// one-peer-at-a-time remainder of small tables keep the element-wise form, which schedules
// their loads better (packed: 8 x 50 M bf16 138.0 -> 141.6, 4 x 25 M 43.8 -> 51.6; f16
// 4 x 25 M 38.8 -> 40.9).  Other dtypes: element-wise Ops::step.
template <int DT, bool PK>
__device__ __attribute__((always_inline)) inline void fold_chunk(typename Ops<DT>::acc_t (&acc)[Ops<DT>::E],
                                                                 typename Ops<DT>::w_t wk, const uint4& v,
                                                                 bool first) {
  using O = Ops<DT>;
  if constexpr ((DT == DLA_BF16 || DT == DLA_F16) && PK) {
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
    if (first) {
      typename O::acc_t x[O::E];
      O::unpack(v, x);
#pragma unroll
      for (int e = 0; e < O::E; ++e) acc[e] = O::zero_mul(x[e]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (DT == DLA_BF16)
        bf16_step2(acc[2 * i], acc[2 * i + 1], wk, w4[i]);
      else
        f16_step2(acc[2 * i], acc[2 * i + 1], wk, w4[i]);
    }
  } else {
    typename O::acc_t x[O::E];
    O::unpack(v, x);
#pragma unroll
    for (int e = 0; e < O::E; ++e) {
      if (first) acc[e] = O::zero_mul(x[e]);
      acc[e] = O::step(acc[e], wk, x[e]);
    }
  }
}

template <int DT, int BS, int CH, bool NT, int SP, bool ACC_IN, bool PK = false, bool PKR = PK>
__device__ __attribute__((always_inline)) inline void fold_tile(
    const void* const* __restrict__ p, const typename Ops<DT>::w_t* __restrict__ w, int n_peers,
    int64_t base0, int64_t n_chunks, uint4* __restrict__ out) {
  using O = Ops<DT>;
  using acc_t = typename O::acc_t;
  constexpr int E = O::E;
  const int64_t base = base0 + threadIdx.x;
  // Lanes past the end of the last (partial) tile load a clamped, valid chunk and
  // skip the store: loads stay unpredicated.
  bool live[CH];
  int64_t idx[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    live[c] = base + c * BS < n_chunks;
    idx[c] = live[c] ? base + c * BS : n_chunks - 1;
  }
  acc_t acc[CH][E];
  int k0 = 0;
  if constexpr (ACC_IN) {
#pragma unroll
    for (int c = 0; c < CH; ++c) O::unpack(out[idx[c]], acc[c]);
  }
  for (; k0 + kGroup <= n_peers; k0 += kGroup) {
    uint4 v[kGroup][CH];
#pragma unroll
    for (int g = 0; g < kGroup; ++g) {
      const uint4* src = static_cast<const uint4*>(p[k0 + g]);
#pragma unroll
      for (int c = 0; c < CH; ++c) v[g][c] = load16<NT>(src + idx[c]);
    }
#pragma unroll
    for (int g = 0; g < kGroup; ++g) {
      const typename O::w_t wk = w[k0 + g];
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        if constexpr (PK) {
          fold_chunk<DT, PK>(acc[c], wk, v[g][c], !ACC_IN && g == 0 && k0 == 0);
        } else {
          acc_t x[E];
          O::unpack(v[g][c], x);
#pragma unroll
          for (int e = 0; e < E; ++e) {
            if (!ACC_IN && g == 0 && k0 == 0) acc[c][e] = O::zero_mul(x[e]);  // fedavg.py:22
            acc[c][e] = O::step(acc[c][e], wk, x[e]);                          // fedavg.py:25
          }
        }
      }
    }
  }
  for (; k0 < n_peers; ++k0) {  // remaining peers (< kGroup), same order
    const uint4* src = static_cast<const uint4*>(p[k0]);
    const typename O::w_t wk = w[k0];
    uint4 v[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = load16<NT>(src + idx[c]);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if constexpr (PKR) {
        fold_chunk<DT, PKR>(acc[c], wk, v[c], !ACC_IN && k0 == 0);
      } else {
        acc_t x[E];
        O::unpack(v[c], x);
#pragma unroll
        for (int e = 0; e < E; ++e) {
          if (!ACC_IN && k0 == 0) acc[c][e] = O::zero_mul(x[e]);
          acc[c][e] = O::step(acc[c][e], wk, x[e]);
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < CH; ++c)
    if (live[c]) store16<SP>(out + idx[c], O::pack(acc[c]));
}

// Ragged tail: elements first..n_elems-1, fewer than one chunk (at most 7), folded by the
// first wave of the block.  The peers' values are gathered lane-parallel (lane l loads
// peer k0+l: 64 loads in flight), transposed through LDS, and lane t folds element t over
// the peers in list order.  A one-lane-per-element loop over the peers waits n_peers
// memory latencies in sequence (12 of the 13 us of a 64-peer x 21 339-element f32 reduce);
// broadcasting every value to every lane instead makes the fold a serial VALU chain of
// n_peers x 7 steps (28 us for one bf16 tail element over 128 peers).
// tile_shift >= 0: the peers are in the tile-interleaved slab layout (dla_wsum_slab_tiled), element j
// of a peer at p[k] + (j >> tile_shift) * tile_stride + (j & (2^tile_shift - 1)).
template <int DT, bool ACC_IN>
__device__ __attribute__((always_inline)) inline void fold_tail(
    const void* const* __restrict__ p, const typename Ops<DT>::w_t* __restrict__ w, int n_peers,
    int64_t first, int64_t n_elems, void* __restrict__ out_v, int tile_shift = -1, int64_t tile_stride = 0) {
  using O = Ops<DT>;
  using acc_t = typename O::acc_t;
  using elem_t = typename O::elem_t;
  constexpr int kMaxTail = O::E - 1;  // a tail is shorter than one 16-byte chunk
  __shared__ elem_t stage[kMaxTail][64];
  const int n_tail = static_cast<int>(n_elems - first);
  if (n_tail <= 0 || threadIdx.x >= 64) return;  // one wave: LDS order within a wave needs no barrier
  const int lane = threadIdx.x;
  const bool owner = lane < n_tail;                // lane t folds tail element t
  elem_t* o = static_cast<elem_t*>(out_v);
  const int64_t mine_j = first + (owner ? lane : 0);
  acc_t acc = ACC_IN ? O::to_acc(o[mine_j]) : acc_t(0);
  for (int k0 = 0; k0 < n_peers; k0 += 64) {
    const int k = k0 + lane < n_peers ? k0 + lane : n_peers - 1;
    const elem_t* src = static_cast<const elem_t*>(p[k]);
    elem_t v[kMaxTail];
#pragma unroll
    for (int t = 0; t < kMaxTail; ++t) {
      const int64_t jj = first + (t < n_tail ? t : n_tail - 1);
      v[t] = src[tile_shift < 0 ? jj : (jj >> tile_shift) * tile_stride + (jj & ((int64_t{1} << tile_shift) - 1))];
    }
#pragma unroll
    for (int t = 0; t < kMaxTail; ++t) stage[t][lane] = v[t];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int m = n_peers - k0 < 64 ? n_peers - k0 : 64;
    if (owner) {
      const elem_t* row = stage[lane];
      for (int l0 = 0; l0 < m; l0 += 8) {  // 8 LDS reads in flight, then 8 ordered steps
        elem_t x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = row[l0 + i];  // all 64 slots are filled (clamped peers)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (l0 + i < m) {
            const acc_t xi = O::to_acc(x[i]);
            if (!ACC_IN && k0 + l0 + i == 0) acc = O::zero_mul(xi);  // fedavg.py:22
            acc = O::step(acc, w[k0 + l0 + i], xi);                  // fedavg.py:25
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // reads done before the next block's writes
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (owner) o[mine_j] = O::from_acc(acc);
}

// ------------------------------------------------ register-stream kernel
// One flat buffer per peer; tiles dealt to workgroups (grid-stride when the grid
// is smaller than the tile count); one extra workgroup folds the ragged tail.
// PKG: packed f16 pair folds in full groups of 8 for an 8-peer table (chosen at launch when
// the pass has 8 peers: the packed group path, even unused, slows the one-peer-at-a-time
// loop of smaller passes; 4 x 25 M f16 39.0 vs 44.3 us).
template <int DT, int KMAX, int BS, int CH, bool NT, int SP, bool ACC_IN, bool PKG = false>
__global__ __launch_bounds__(BS) void wsum_stream_kernel(
    const PeerTable<typename Ops<DT>::w_t, KMAX> tab, int n_peers, int64_t n_chunks,
    int64_t n_elems, void* __restrict__ out_v) {
  const int64_t tile_chunks = static_cast<int64_t>(BS) * CH;
  const int64_t n_tiles = (n_chunks + tile_chunks - 1) / tile_chunks;
  // A ragged tail gets the grid's last workgroup to itself, so it overlaps the tiles.
  const bool has_tail = n_elems > n_chunks * Ops<DT>::E;
  const int64_t main_grid = static_cast<int64_t>(gridDim.x) - (has_tail ? 1 : 0);
  if (has_tail && blockIdx.x == main_grid) {
    fold_tail<DT, ACC_IN>(tab.p, tab.w, n_peers, n_chunks * Ops<DT>::E, n_elems, out_v);
    return;
  }
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += main_grid)
    fold_tile<DT, BS, CH, NT, SP, ACC_IN, (KMAX > 8 || PKG), (KMAX > 8)>(tab.p, tab.w, n_peers, tile * tile_chunks, n_chunks,
                                                       static_cast<uint4*>(out_v));
}

// ------------------------------------------------ peer-major big-tile kernel
// The north-star shape (<= 8 peers, large P): one wave owns a "big tile" of 64 * BT
// contiguous 16-byte chunks (16 KiB of output at BT = 16).  It streams peer 0's 16 KiB,
// then peer 1's, ... (the loads of peer k+1 are in flight while peer k is folded, and the
// other waves of the CU cover the rest), then writes its 16 KiB.  Per element the fold is
// the same list-order sequence as fold_tile.  Measured on MI355X (profiles/phase_probe.py):
// 8 x 25 M fp32 133.2 us against 138.2 us for the 1-chunk-per-lane stream; BT = 8 gives
// 141.9 us, BT = 24 / 32 lose occupancy (164.8 / 185.6 us).  The pattern's own ceiling on
// the same box: 8-stream read alone 116.4-117.5 us + the 100 MB sc1 write alone 14.8 us.
template <int DT, int NP, int BT>
__device__ __attribute__((always_inline)) inline void fold_big_tile(
    const void* const* __restrict__ p, const typename Ops<DT>::w_t* __restrict__ w, int64_t base,
    int64_t n_chunks, uint4* __restrict__ out) {
  using O = Ops<DT>;
  using acc_t = typename O::acc_t;
  constexpr int E = O::E;
  // chunk c of this lane: base + c * 64 (full tiles only: one base plus immediate offsets)
  auto at = [&](int c) -> int64_t { return base + c * 64; };
  // pointers and weights into registers first: the compiler barrier below must not force
  // them to be re-read from the kernel-argument segment
  const u32x4* src[NP];
  typename O::w_t wv[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    src[k] = static_cast<const u32x4*>(p[k]);
    wv[k] = w[k];
  }
  acc_t acc[BT][E];
  u32x4 a[BT], b[BT];
#pragma unroll
  for (int c = 0; c < BT; ++c) a[c] = __builtin_nontemporal_load(src[0] + at(c));
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    if (k + 1 < NP) {
#pragma unroll
      for (int c = 0; c < BT; ++c) b[c] = __builtin_nontemporal_load(src[k + 1] + at(c));
    }
    asm volatile("" ::: "memory");  // peer k+2's loads stay below peer k's fold: two buffers
    const typename O::w_t wk = wv[k];
#pragma unroll
    for (int c = 0; c < BT; ++c) {
      acc_t x[E];
      O::unpack(make_uint4(a[c].x, a[c].y, a[c].z, a[c].w), x);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (k == 0) acc[c][e] = O::zero_mul(x[e]);  // fedavg.py:22
        acc[c][e] = O::step(acc[c][e], wk, x[e]);   // fedavg.py:25
      }
    }
    if (k + 1 < NP) {
#pragma unroll
      for (int c = 0; c < BT; ++c) a[c] = b[c];
    }
  }
#pragma unroll
  for (int c = 0; c < BT; ++c)
    store16<2>(out + at(c), O::pack(acc[c]));
}

// NP: the exact peer count, so the peer loop is fully static.  Workgroups [0, n_big) fold
// big tiles; the next n_seg_wg workgroups fold chunks [n_big * kTile, n_chunks) as 64-chunk
// stream segments, strided over those workgroups; one more folds the ragged tail, if any.
// Default launch: n_big = every full tile and one segment workgroup for the partial last
// tile.  Balanced launch (variant 17): n_big = whole rounds of resident big tiles only, and
// the rest spread over up to one round of segment workgroups, so a partial last round does
// not leave most of the chip idle.
template <int DT, int NP, int BT, int KMAX = 8>
__global__ __launch_bounds__(64) void wsum_bigtile_kernel(const PeerTable<typename Ops<DT>::w_t, KMAX> tab,
                                                          int64_t n_chunks, int64_t n_elems,
                                                          int64_t n_big, int64_t n_seg_wg,
                                                          void* __restrict__ out_v) {
  constexpr int64_t kTile = 64 * BT;
  const int64_t b = blockIdx.x;
  uint4* out = static_cast<uint4*>(out_v);
  if (b < n_big) {
    // Written as a grid-stride loop although it runs once per workgroup: inside a loop hipcc
    // keeps the two-buffer schedule (peer k+1's 16 loads in flight while peer k folds, ~16-20
    // loads outstanding, <= 256 VGPRs); as straight-line code it waits for every load before
    // each fold and spills the peers' data into AGPRs.
    for (int64_t t = b; t < n_big; t += gridDim.x)
      fold_big_tile<DT, NP, BT>(tab.p, tab.w, t * kTile + threadIdx.x, n_chunks, out);
    return;
  }
  if (b < n_big + n_seg_wg) {  // the chunks after the big tiles, as 64-chunk segments
    for (int64_t t0 = n_big * kTile + (b - n_big) * 64; t0 < n_chunks; t0 += n_seg_wg * 64)
      fold_tile<DT, 64, 1, true, 2, false>(tab.p, tab.w, NP, t0, n_chunks, out);
    return;
  }
  fold_tail<DT, false>(tab.p, tab.w, NP, n_chunks * Ops<DT>::E, n_elems, out_v);  // no-op without a tail
}

// ------------------------------------------------ word-per-lane ("wide") kernel
// For a small share reduced over many peers the 16-byte register stream has too few lanes
// to cover the memory latency: each lane waits for its groups of 8 peers one after the
// other (128 peers x 85 354 fp32: 16 waits per lane, 24 us; 9 us here).  Here each lane owns
// one 4-byte word (8 for f64) and issues the loads of G peers at once before folding them
// in list order, so a pass of up to G peers costs about one memory latency, with 4x the
// lanes of the 16-byte stream.  Same fold as fold_tile.
template <typename W>
__device__ inline W load_word_nt(const W* p) {
  return __builtin_nontemporal_load(p);  // global_load_dword[x2] ... nt
}
__device__ inline void store_word_sc1(uint32_t* p, uint32_t v) {
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ inline void store_word_sc1(u32x2* p, u32x2 v) {
  asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

// Fold G loaded words in list order.  FULL (every slot a live peer): no per-peer
// conditions, so the weights load as one batch; otherwise peers g >= m are skipped.
template <int DT, int G, bool FULL, bool ACC_IN>
__device__ __attribute__((always_inline)) inline void fold_words(
    const typename Ops<DT>::word_t (&v)[G], const typename Ops<DT>::w_t* __restrict__ w, int m, bool first_round,
    typename Ops<DT>::acc_t (&acc)[Ops<DT>::WE]) {
  using O = Ops<DT>;
  using acc_t = typename O::acc_t;
  typename O::w_t wk[G];
#pragma unroll
  for (int g = 0; g < G; ++g) wk[g] = w[g];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (FULL || g < m) {
      if constexpr (DT == DLA_BF16) {
        // both bf16 elements of the word at once: v_pk_mul_f32 / v_pk_add_f32 and one
        // v_cvt_pk_bf16_f32 per rounding (same per-element arithmetic as Ops::step)
        if (!ACC_IN && g == 0 && first_round) {
          acc_t x[2];
          O::unpack_w(v[g], x);
          acc[0] = O::zero_mul(x[0]);  // fedavg.py:22
          acc[1] = O::zero_mul(x[1]);
        }
        bf16_step2(acc, wk[g], v[g]);  // fedavg.py:25
      } else if constexpr (DT == DLA_F16) {  // likewise, v_cvt_pk_f16_f32 per rounding
        if (!ACC_IN && g == 0 && first_round) {
          acc_t x[2];
          O::unpack_w(v[g], x);
          acc[0] = O::zero_mul(x[0]);  // fedavg.py:22
          acc[1] = O::zero_mul(x[1]);
        }
        f16_step2(acc[0], acc[1], wk[g], v[g]);  // fedavg.py:25
      } else {
        acc_t x[O::WE];
        O::unpack_w(v[g], x);
#pragma unroll
        for (int e = 0; e < O::WE; ++e) {
          if (!ACC_IN && g == 0 && first_round) acc[e] = O::zero_mul(x[e]);  // fedavg.py:22
          acc[e] = O::step(acc[e], wk[g], x[e]);                              // fedavg.py:25
        }
      }
    }
  }
}

template <int DT, int KMAX, int G, bool ACC_IN>
__global__ __launch_bounds__(64) void wsum_wide_kernel(
    const PeerTable<typename Ops<DT>::w_t, KMAX> tab, int n_peers, int64_t n_words,
    int64_t n_elems, void* __restrict__ out_v) {
  using O = Ops<DT>;
  using acc_t = typename O::acc_t;
  using word_t = typename O::word_t;
  constexpr int WE = O::WE;
  const int64_t main_grid = (n_words + 63) / 64;
  if (blockIdx.x >= main_grid) {  // the ragged-tail workgroup (at most WE - 1 elements)
    fold_tail<DT, ACC_IN>(tab.p, tab.w, n_peers, n_words * WE, n_elems, out_v);
    return;
  }
  {
    const int64_t j = static_cast<int64_t>(blockIdx.x) * 64 + threadIdx.x;
    const bool live = j < n_words;
    const int64_t i = live ? j : n_words - 1;  // clamped: loads stay unpredicated
    word_t* out = static_cast<word_t*>(out_v);
    acc_t acc[WE];
    if constexpr (ACC_IN) O::unpack_w(out[i], acc);
    // Rounds unrolled: every table index is a compile-time constant, so the pointers and
    // weights arrive in batched s_load_dwordx16 reads instead of one scalar load and wait
    // per peer (which cost ~5 us per 64-peer round before).
#pragma unroll
    for (int r = 0; r < (KMAX + G - 1) / G; ++r) {
      const int k0 = r * G;
      if (k0 >= n_peers) break;
      word_t v[G];
      if (k0 + G <= n_peers) {  // full round: its own path (64 x 21 339 fp32: 5.1 -> 4.4 us)
#pragma unroll
        for (int g = 0; g < G; ++g) v[g] = load_word_nt(static_cast<const word_t*>(tab.p[k0 + g]) + i);
        fold_words<DT, G, true, ACC_IN>(v, tab.w + k0, G, k0 == 0, acc);
      } else {
        // partial round: slots past the last peer reload it (cached; branch-free issue).
        // Predicating those loads instead measured slower: 100 x 200 K fp32 14.7 vs 13.0 us.
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int k = k0 + g < n_peers ? k0 + g : n_peers - 1;
          v[g] = load_word_nt(static_cast<const word_t*>(tab.p[k]) + i);
        }
        fold_words<DT, G, false, ACC_IN>(v, tab.w + k0, n_peers - k0, k0 == 0, acc);
      }
    }
    if (live) store_word_sc1(out + i, O::pack_w(acc));
  }
}

// ------------------------------------------------ vector-per-lane ("wide-VW") kernel
// The word-per-lane kernel with VW dwords per lane per load (8 or 16 bytes: dwordx2 / dwordx4):
// G peers' loads in flight per lane, then the list-order fold of each dword (bf16 / f16: two
// elements per dword through bf16_step2 / f16_step2; f32: one).  Same fold, same rounding
// sequence as wsum_wide_kernel; 2-4x fewer load instructions per byte.
template <int VW> struct VecOf;
template <> struct VecOf<2> { using T = u32x2; };
template <> struct VecOf<4> { using T = u32x4; };

template <int DT>
__device__ __attribute__((always_inline)) inline void fold_dword(typename Ops<DT>::acc_t* acc,
                                                                 typename Ops<DT>::w_t wk, uint32_t word, bool first) {
  using O = Ops<DT>;
  if (first) {
    typename O::acc_t x[O::WE];
    O::unpack_w(word, x);
#pragma unroll
    for (int e = 0; e < O::WE; ++e) acc[e] = O::zero_mul(x[e]);  // fedavg.py:22
  }
  if constexpr (DT == DLA_BF16) {
    bf16_step2(acc[0], acc[1], wk, word);  // fedavg.py:25, both elements
  } else if constexpr (DT == DLA_F16) {
    f16_step2(acc[0], acc[1], wk, word);
  } else {
    acc[0] = O::step(acc[0], wk, __uint_as_float(word));
  }
}

__device__ inline void store_vec_sc1(u32x2* p, u32x2 v) {
  asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ inline void store_vec_sc1(u32x4* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// A peer pointer as a global-address-space pointer: global_load (not flat_load) whatever the pointer
// came from (the kernel-argument table is promoted to global by the backend; a pointer read from a
// device-side table is not).
template <class T>
__device__ __attribute__((always_inline)) inline const __attribute__((address_space(1))) T* gptr(const void* p) {
  return (const __attribute__((address_space(1))) T*)(p);
}

// TAB: anything with tab.p[k] (peer pointers) and tab.w[k] (op-math weights): the kernel-argument
// PeerTable, or a PeerRef into a device-side pointer table (wsum_multi_vec_kernel).
template <int DT, int KMAX, int G, int VW, bool FULL, bool ACC_IN, class TAB>
__device__ __attribute__((always_inline)) inline void vec_round(
    const TAB& tab, int k0, int m, bool first_round, int64_t a,
    typename Ops<DT>::acc_t (&acc)[VW][Ops<DT>::WE]) {
  using V = typename VecOf<VW>::T;
  V v[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    // partial round: slots past the last peer reload it (cached; branch-free issue)
    const int k = FULL || g < m ? k0 + g : k0 + m - 1;
    v[g] = __builtin_nontemporal_load(gptr<V>(tab.p[k]) + a);
  }
  typename Ops<DT>::w_t wk[G];
#pragma unroll
  for (int g = 0; g < G; ++g) wk[g] = tab.w[k0 + g];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (FULL || g < m) {
#pragma unroll
      for (int d = 0; d < VW; ++d) fold_dword<DT>(acc[d], wk[g], v[g][d], !ACC_IN && first_round && g == 0);
    }
  }
}

// The m < G peers of a last round as rounds of G/2, G/4, ..., 1 peers (each full, of compile-time
// size, in list order): no slot reloads a peer, so a 2-peer pass issues 2 loads per lane, not G.
// Against the partial round that reloaded the last peer into the spare slots (r02 A/B,
// profiles/r02v_ab_tail.log, tiled slab, us): 2 x 25 M f32 72.4 -> 44.5, 4 x 25 M f32 82.3 ->
// 73.8, 12 x 11.2 M f32 88.5 -> 84.8, 20 x 5 M f32 73.1 -> 61.0, 48 x 1.23 M f32 39.0 -> 35.0,
// 100 x 2.66 M bf16 83.3 -> 79.6, 3 x 50 M bf16 77.4 -> 64.0 (separate buffers alike).
template <int DT, int KMAX, int G, int VW, bool ACC_IN, class TAB>
__device__ __attribute__((always_inline)) inline void vec_tail(
    const TAB& tab, int k0, int m, bool first_round, int64_t a,
    typename Ops<DT>::acc_t (&acc)[VW][Ops<DT>::WE]) {
  if constexpr (G > 1) {
    constexpr int H = G / 2;
    if (m >= H) {
      vec_round<DT, KMAX, H, VW, true, ACC_IN>(tab, k0, H, first_round, a, acc);
      k0 += H;
      m -= H;
      first_round = false;
    }
    vec_tail<DT, KMAX, H, VW, ACC_IN>(tab, k0, m, first_round, a, acc);
  }
}

// TILED: the peers are rows of a tile-interleaved slab (dla_wsum_slab_tiled): vector i of a peer at
// p[k] + (i >> tshift_v) * tstride_v + (i & (2^tshift_v - 1)); the output stays contiguous.
// PLAIN_ST: plain (L2 write-back) output stores instead of sc1 — faster when the output is small
// and many peers are read per element, slower for large outputs (vec_store_policy).
template <int DT, int KMAX, int G, int VW, bool ACC_IN, bool TILED = false, bool PLAIN_ST = false>
__global__ __launch_bounds__(64) void wsum_vec_kernel(
    const PeerTable<typename Ops<DT>::w_t, KMAX> tab, int n_peers, int64_t n_vecs,
    int64_t n_elems, void* __restrict__ out_v, int tshift_v = 0, int64_t tstride_v = 0, int tshift_e = -1,
    int64_t tstride_e = 0) {
  static_assert(DT != DLA_F64, "dword folds: f32 / bf16 / f16");
  using O = Ops<DT>;
  using acc_t = typename O::acc_t;
  using V = typename VecOf<VW>::T;
  constexpr int WE = O::WE;               // elements per dword
  const int64_t main_grid = (n_vecs + 63) / 64;
  if (blockIdx.x >= main_grid) {  // the ragged-tail workgroup (< VW * WE elements)
    fold_tail<DT, ACC_IN>(tab.p, tab.w, n_peers, n_vecs * VW * WE, n_elems, out_v, TILED ? tshift_e : -1,
                          tstride_e);
    return;
  }
  const int64_t j = static_cast<int64_t>(blockIdx.x) * 64 + threadIdx.x;
  const bool live = j < n_vecs;
  const int64_t i = live ? j : n_vecs - 1;  // clamped: loads stay unpredicated
  const int64_t a = TILED ? (i >> tshift_v) * tstride_v + (i & ((int64_t{1} << tshift_v) - 1)) : i;
  V* out = static_cast<V*>(out_v);
  acc_t acc[VW][WE];
  if constexpr (ACC_IN) {
    const V o = out[i];
#pragma unroll
    for (int d = 0; d < VW; ++d) O::unpack_w(o[d], acc[d]);
  }
#pragma unroll
  for (int r = 0; r < (KMAX + G - 1) / G; ++r) {
    const int k0 = r * G;
    if (k0 >= n_peers) break;
    if (k0 + G <= n_peers) {  // full round: its own unpredicated path (as wsum_wide_kernel)
      vec_round<DT, KMAX, G, VW, true, ACC_IN>(tab, k0, G, r == 0, a, acc);
    } else {
      vec_tail<DT, KMAX, G, VW, ACC_IN>(tab, k0, n_peers - k0, r == 0, a, acc);
      break;
    }
  }
  if (live) {
    V o;
#pragma unroll
    for (int d = 0; d < VW; ++d) o[d] = O::pack_w(acc[d]);
    if constexpr (PLAIN_ST)
      out[i] = o;
    else
      store_vec_sc1(out + i, o);
  }
}

// ------------------------------------------------ many-peer multi-tensor kernel
// dla_wsum_multi_table: every 16-byte aligned parameter tensor of a round (fedavg.py:24 walks them
// one by one) over a pass of up to 128 peers in ONE launch.  The (tensor x peer) pointer table does
// not fit the kernel-argument block (128 google_speech ResNet-34 models: 14 080 pointers), so it
// travels to the device as one table per call (upload_table: a copy kernel, or a side-stream copy
// that overlaps the kernel before it).  Workgroup b finds its
// tensor from the tensors' first workgroups (uniform: scalar loads), then folds 64 vectors of it
// exactly as wsum_vec_kernel does (8 bytes per lane, G peers' loads in flight, list order); a tensor
// with a ragged tail has one more workgroup, which runs fold_tail.  A launch covers up to 256 tensors.
struct MultiSeg {
  int64_t wg_begin;         // first workgroup of this tensor in the launch
  int64_t n_vecs;           // whole 8-byte vectors of the tensor
  int64_t n_elems;
  void* out;
  const void* const* ptrs;  // this tensor's row of the device pointer table (n_peers entries)
};

// The tensors' first workgroups for the two-level search: coarse[q] = fine[16 q]; entries past the
// last tensor are INT32_MAX.  Workgroup b counts the coarse entries <= b (one s_load_dwordx16), then
// the fine entries <= b in that block of 16 (one more): two dependent scalar loads instead of the
// eight of a binary search over 256 tensors.
struct MultiIndex {
  int32_t coarse[16];
  int32_t fine[256];
};
constexpr int kMultiTensorsPerLaunch = 256;

// One row of the device pointer table, read through the constant address space: the table is never
// written while the kernel runs, and uniform reads of it then become scalar loads (s_load_dwordx16
// batches, as from the kernel-argument table) instead of a vector load per pointer per lane.
typedef const void* PeerPtr;
typedef const __attribute__((address_space(4))) PeerPtr* ConstPeerTab;
typedef const __attribute__((address_space(4))) int32_t* ConstI32;

template <typename W>
struct PeerRef {  // the PeerTable interface (tab.p[k], tab.w[k]) over one row of the device table
  ConstPeerTab p;
  const W* __restrict__ w;
};

// Workgroup b's tensor: count the coarse entries <= b (one s_load_dwordx16 batch), then the fine
// entries <= b in that block of 16 (a second one).  (A binary search over the records' wg_begin — eight
// dependent scalar loads for 256 tensors — measured the same, profiles/r03d/: the lookup is not what
// bounds this kernel.)
__device__ __attribute__((always_inline)) inline int multi_segment(const MultiIndex* idx, int b) {
  const ConstI32 cz = (ConstI32)(idx->coarse);
  int c = 0;
#pragma unroll
  for (int q = 1; q < 16; ++q) c += cz[q] <= b ? 1 : 0;
  const ConstI32 fz = (ConstI32)(idx->fine + 16 * c);
  int t = 16 * c;
#pragma unroll
  for (int q = 1; q < 16; ++q) t += fz[q] <= b ? 1 : 0;
  return t;
}

template <typename W, int KMAX>
struct WeightTable {
  W w[KMAX];
};

template <int DT, int KMAX, int G, bool ACC_IN, bool PLAIN_ST>
__global__ __launch_bounds__(64) void wsum_multi_vec_kernel(const MultiIndex* __restrict__ idx,
                                                            const MultiSeg* __restrict__ segs, int n_seg, int k0,
                                                            int n_peers,
                                                            const WeightTable<typename Ops<DT>::w_t, KMAX> wt) {
  static_assert(DT != DLA_F64, "dword folds: f32 / bf16 / f16");
  using O = Ops<DT>;
  using acc_t = typename O::acc_t;
  constexpr int VW = 2;
  using V = typename VecOf<VW>::T;
  constexpr int WE = O::WE;
  const int64_t b = blockIdx.x;
  const int lo = multi_segment(idx, static_cast<int>(blockIdx.x));
  const int64_t n_vecs = segs[lo].n_vecs;
  const int64_t local = b - segs[lo].wg_begin;
  const PeerRef<typename O::w_t> tab{(ConstPeerTab)(segs[lo].ptrs + k0), wt.w};
  void* const out_v = segs[lo].out;
  if (local >= (n_vecs + 63) / 64) {  // this tensor's ragged-tail workgroup
    fold_tail<DT, ACC_IN>(segs[lo].ptrs + k0, tab.w, n_peers, n_vecs * VW * WE, segs[lo].n_elems, out_v);
    return;
  }
  const int64_t j = local * 64 + threadIdx.x;
  const bool live = j < n_vecs;
  const int64_t i = live ? j : n_vecs - 1;  // clamped: loads stay unpredicated
  V* out = static_cast<V*>(out_v);
  __attribute__((address_space(1))) V* gout = (__attribute__((address_space(1))) V*)out_v;  // global_* access
  acc_t acc[VW][WE];
  if constexpr (ACC_IN) {
    const V o = gout[i];
#pragma unroll
    for (int d = 0; d < VW; ++d) O::unpack_w(o[d], acc[d]);
  }
#pragma unroll
  for (int r = 0; r < (KMAX + G - 1) / G; ++r) {
    const int r0 = r * G;
    if (r0 >= n_peers) break;
    if (r0 + G <= n_peers) {
      vec_round<DT, KMAX, G, VW, true, ACC_IN>(tab, r0, G, r == 0, i, acc);
    } else {
      vec_tail<DT, KMAX, G, VW, ACC_IN>(tab, r0, n_peers - r0, r == 0, i, acc);
      break;
    }
  }
  if (live) {
    V o;
#pragma unroll
    for (int d = 0; d < VW; ++d) o[d] = O::pack_w(acc[d]);
    if constexpr (PLAIN_ST)
      gout[i] = o;
    else
      store_vec_sc1(out + i, o);
  }
}

// ------------------------------------------------ multi-tensor kernel
// Up to MAXSEG parameter tensors ("segments") of one model in ONE launch
// (fedavg.py:24 walks them one by one).  Workgroup b finds its segment from the
// cumulative tile counts (a short uniform scan: scalar code), then folds one CH=1
// tile of it; the first tile of each segment also folds that segment's tail.
template <typename W, int NP, int MAXSEG>
struct SegTable {
  const void* p[MAXSEG][NP];
  void* out[MAXSEG];
  int64_t tile_end[MAXSEG];  // cumulative tiles through segment s
  int64_t n_elems[MAXSEG];
  W w[NP];
};

template <int DT, int NP, int MAXSEG, int SP>
__global__ __launch_bounds__(kBlock) void wsum_multi_kernel(
    const SegTable<typename Ops<DT>::w_t, NP, MAXSEG> tab, int n_seg, int n_peers) {
  const int64_t b = blockIdx.x;
  int s = 0;
  while (s < n_seg - 1 && tab.tile_end[s] <= b) ++s;
  const int64_t tile = b - (s ? tab.tile_end[s - 1] : 0);
  const int64_t n_elems = tab.n_elems[s];
  const int64_t n_chunks = n_elems / Ops<DT>::E;
  if (tile * kBlock < n_chunks)
    fold_tile<DT, kBlock, 1, true, SP, false, (NP > 8 || DT == DLA_F16), (NP > 8)>(tab.p[s], tab.w, n_peers, tile * kBlock, n_chunks,
                                      static_cast<uint4*>(tab.out[s]));
  if (tile == 0) fold_tail<DT, false>(tab.p[s], tab.w, n_peers, n_chunks * Ops<DT>::E, n_elems, tab.out[s]);
}

// ------------------------------------------------ teacher-logit mean (§8 f4)
// scripts/distill.py:124-129: torch.mean(torch.stack(preds), dim=0) = sum / N.  Contract:
// acc = +0; acc = acc + p_k in list order (op-math = storage type, F32/F64 only); the last
// pass divides by N (correctly rounded).  torch's own CPU/GPU sum order is an
// implementation detail (vectorised columns sequential, tail columns and N > 16 cascaded),
// so parity with torch.mean is within a stated tolerance; with the sequential oracle it is
// bit-exact.  One 16-byte chunk per lane, 64-thread workgroups.
template <int DT, int KMAX, bool ACC_IN, bool ALIGNED>
__global__ __launch_bounds__(64) void mean_kernel(const PeerTable<typename Ops<DT>::w_t, KMAX> tab, int n_peers,
                                                  int64_t n_chunks, int64_t n_elems, void* __restrict__ out_v,
                                                  typename Ops<DT>::acc_t divisor, int divide) {
  using O = Ops<DT>;
  using acc_t = typename O::acc_t;
  using elem_t = typename O::elem_t;
  constexpr int E = O::E;
  static_assert(DT == DLA_F32 || DT == DLA_F64, "mean: f32/f64 only");
  if constexpr (ALIGNED) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * 64 + threadIdx.x;
    if (i < n_chunks) {
      uint4* out = static_cast<uint4*>(out_v);
      acc_t acc[E];
      if constexpr (ACC_IN) {
        O::unpack(out[i], acc);
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] = acc_t(0);
      }
      int k = 0;
      for (; k + kGroup <= n_peers; k += kGroup) {
        uint4 v[kGroup];
#pragma unroll
        for (int g = 0; g < kGroup; ++g) v[g] = load16<true>(static_cast<const uint4*>(tab.p[k + g]) + i);
#pragma unroll
        for (int g = 0; g < kGroup; ++g) {
          acc_t x[E];
          O::unpack(v[g], x);
#pragma unroll
          for (int e = 0; e < E; ++e) acc[e] = acc[e] + x[e];
        }
      }
      for (; k < n_peers; ++k) {
        acc_t x[E];
        O::unpack(load16<true>(static_cast<const uint4*>(tab.p[k]) + i), x);
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] = acc[e] + x[e];
      }
      if (divide) {
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] = acc[e] / divisor;
      }
      store16<2>(out + i, O::pack(acc));
    }
  }
  // ragged tail (aligned) or everything (unaligned): one element per lane
  const int64_t j0 = ALIGNED ? n_chunks * E : 0;
  const int64_t stride = ALIGNED ? 64 : static_cast<int64_t>(gridDim.x) * 64;
  const int64_t start = ALIGNED ? (blockIdx.x == 0 ? j0 + threadIdx.x : n_elems)
                                : static_cast<int64_t>(blockIdx.x) * 64 + threadIdx.x;
  for (int64_t j = start; j < n_elems; j += stride) {
    elem_t* o = static_cast<elem_t*>(out_v);
    acc_t acc = ACC_IN ? O::to_acc(o[j]) : acc_t(0);
    for (int k = 0; k < n_peers; ++k) acc = acc + O::to_acc(static_cast<const elem_t*>(tab.p[k])[j]);
    if (divide) acc = acc / divisor;
    o[j] = O::from_acc(acc);
  }
}

// ---------------------------------------------------- scalar kernel (unaligned)
// Any alignment; one element per lane, grid-stride.  Used only when a buffer is
// not 16-byte aligned (e.g. an odd-offset view).
template <int DT, int KMAX, bool ACC_IN>
__global__ __launch_bounds__(kBlock) void wsum_scalar_kernel(
    const PeerTable<typename Ops<DT>::w_t, KMAX> tab, int n_peers, int64_t n_elems,
    void* __restrict__ out_v) {
  using O = Ops<DT>;
  using acc_t = typename O::acc_t;
  using elem_t = typename O::elem_t;
  elem_t* o = static_cast<elem_t*>(out_v);
  for (int64_t j = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; j < n_elems;
       j += static_cast<int64_t>(gridDim.x) * kBlock) {
    acc_t acc = ACC_IN ? O::to_acc(o[j]) : acc_t(0);
    for (int k = 0; k < n_peers; ++k) {
      const acc_t x = O::to_acc(static_cast<const elem_t*>(tab.p[k])[j]);
      if (!ACC_IN && k == 0) acc = O::zero_mul(x);
      acc = O::step(acc, tab.w[k], x);
    }
    o[j] = O::from_acc(acc);
  }
}

// ------------------------------------------------- mixed-dtype kernel (peers of several dtypes)
// fedavg.py:25 `c1.add_(w * p1)` when peer k's parameter has another dtype than models[0]'s (the
// centre's): torch computes w * p1 in p1's op-math and rounds it to p1's dtype, then adds in the
// op-math of the PROMOTED type (f64 if either side is f64, else f32) and rounds the sum to the
// centre's dtype; a double sum lands in a 16-bit centre through float (c10::BFloat16 / c10::Half
// take a float).  The running sum is carried as a double holding a value of the centre's dtype
// exactly.  One element per lane; the dtype switch is uniform across the wave (per peer).  A rare
// path (mixed rounds do not occur at the reference's call sites), so it is plain and scalar.
struct MixedTable {
  const void* p[kMaxPeersPerPass];
  double w[kMaxPeersPerPass];
  int8_t dt[kMaxPeersPerPass];
};

__device__ inline double mixed_load(const void* p, int dt, int64_t j) {
  switch (dt) {
    case DLA_F32: return static_cast<double>(static_cast<const float*>(p)[j]);
    case DLA_BF16: return static_cast<double>(bf16_bits_to_f(static_cast<const uint16_t*>(p)[j]));
    case DLA_F16: return static_cast<double>(half_bits_to_f(static_cast<const uint16_t*>(p)[j]));
    default: return static_cast<const double*>(p)[j];
  }
}

// an f32 op-math result rounded RNE to dtype dt (F32, BF16 or F16), as f32
__device__ inline float mixed_round32(float f, int dt) {
  return dt == DLA_BF16 ? round_bf16(pin(f)) : dt == DLA_F16 ? round_f16(f) : f;
}

// an f64 op-math result rounded to dtype dt (to 16-bit dtypes through float, as torch casts)
__device__ inline double mixed_round64(double d, int dt) {
  if (dt == DLA_F64) return d;
  return static_cast<double>(mixed_round32(pin(static_cast<float>(d)), dt));
}

__device__ inline void mixed_store(void* p, int dt, int64_t j, double v) {
  switch (dt) {
    case DLA_F32: static_cast<float*>(p)[j] = static_cast<float>(v); break;
    case DLA_BF16:  // v is a bf16 value: its f32 pattern's high half is the bf16
      static_cast<uint16_t*>(p)[j] = static_cast<uint16_t>(__float_as_uint(static_cast<float>(v)) >> 16);
      break;
    case DLA_F16: static_cast<uint16_t*>(p)[j] = static_cast<uint16_t>(f_to_half_bits(static_cast<float>(v))); break;
    default: static_cast<double*>(p)[j] = v; break;
  }
}

template <bool ACC_IN>
__global__ __launch_bounds__(kBlock) void wsum_mixed_kernel(const MixedTable tab, int n_peers, int out_dt,
                                                            int64_t n_elems, void* __restrict__ out) {
  for (int64_t j = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; j < n_elems;
       j += static_cast<int64_t>(gridDim.x) * kBlock) {
    double acc = ACC_IN ? mixed_load(out, out_dt, j) : 0.0;
    for (int k = 0; k < n_peers; ++k) {
      const int dk = tab.dt[k];
      const double x = mixed_load(tab.p[k], dk, j);
      if (!ACC_IN && k == 0)  // fedavg.py:22 p.mul_(0) on models[0]'s own values (peer 0 has out_dt)
        acc = out_dt == DLA_F64 ? x * 0.0 : static_cast<double>(static_cast<float>(x) * 0.0f);
      const double prod = dk == DLA_F64 ? tab.w[k] * x
                                        : static_cast<double>(mixed_round32(
                                              static_cast<float>(tab.w[k]) * static_cast<float>(x), dk));
      acc = (out_dt == DLA_F64 || dk == DLA_F64)
                ? mixed_round64(acc + prod, out_dt)
                : static_cast<double>(mixed_round32(static_cast<float>(acc) + static_cast<float>(prod), out_dt));
    }
    mixed_store(out, out_dt, j, acc);
  }
}

// ------------------------------------------------------------------ launching

struct Launch {
  int variant;      // 1 plain/plain, 2 nt/plain, 4 nt/sc1 (load/store cache policy); 8 wide kernel
  bool auto_kernel; // variant not forced: the wide kernel may be picked by shape (use_wide)
  int block;        // 64 or 256 threads; 0 = pick (shape_for)
  int chunks;       // 1, 2, 4; 0 = pick (shape_for)
  int grid_blocks;  // 0 = one workgroup per tile
};

// Workgroup shape by dtype, peer count and size (interleaved A/B on MI355X, r01 sweeps):
//  * default: 64-thread workgroups, 1 chunk per lane — the most, smallest workgroups.
//    8 x 25 M fp32: 6.50 vs 6.39 TB/s for 256 x 4; 16 x 21.3 M fp32 6.44 vs 6.24;
//    128 x 21.3 M bf16 (google_speech) 6.48 vs 6.27.
//  * 16-bit dtypes with <= 16 peers: 256 x 4 (each chunk carries 8 elements of VALU work;
//    more chunks per lane keep more bytes in flight): 8 x 50 M bf16 6.65 vs 6.38 TB/s —
//    while that still leaves >= 2048 tiles (8 per CU).
void shape_for(int64_t n_chunks, int n_peers, int elems_per_chunk, int* block, int* chunks) {
  constexpr int64_t kMinTiles = 2048;
  if (elems_per_chunk == 8 && n_peers <= 16 && n_chunks >= kMinTiles * 256 * 4) {
    *block = 256;
    *chunks = 4;
    return;
  }
  *block = 64;
  *chunks = 1;
}

// The wide kernel (one word per lane, up to 64 peers in flight) is picked for
//  * small shares over more than 8 peers, where the 16-byte stream leaves the chip mostly idle
//    while each lane waits group after group (64 x 21 339 fp32, configs[3]: 12.8 -> 5.1 us;
//    128 x 85 354 fp32: 29.3 -> 9.2 us);
//  * 16-bit dtypes over more than 32 peers at any size (128 x 2 662 045 bf16, configs[4]'s
//    per-GPU share: 115.1 -> 111.4 us; 128 x 665 511 bf16: 35.4 -> 32.3 us).
// f32 shares of >= 128 K chunks keep the stream (32 x 1 690 046: 34.5 vs 35.8 us; 64 x 1 233 086:
// 48.2 vs 52.4 us).  Interleaved A/B on MI355X: profiles/r01_ab_wide*.log.
// Passes of more than 8 peers in fp32 / bf16 / f16 take the vector-per-lane kernel (8 bytes per
// lane per load): 32 peers in flight per lane for passes of >= 32 peers (variant 9), else 16
// (variant 12: a 32-slot round would reload the last peer into every unused slot).  Interleaved
// A/B on MI355X against the word-per-lane kernel / 16-byte stream this replaces (us,
// profiles/r02b_ab_vec.log): 128 x 2 662 045 bf16 106.2 vs 109.9, 128 x 21.3 M bf16 840.5 vs
// 857.6, 128 x 665 511 bf16 27.6 vs 30.4, 16 x 21.3 M bf16 112.4 vs 118.9, 32 x 1 690 046 f32
// 33.4 vs 34.4, 64 x 1 233 086 f32 48.4 vs 48.4, 128 x 85 354 f32 10.9 vs 11.1.
int vec_variant(int n_peers) { return n_peers >= 32 ? 9 : 12; }

// Plain output stores (variant 21) for passes of >= 32 peers whose output is at most 8 MiB (it
// then stays in the 8 x 4 MB of L2 until written back).  r02 interleaved A/B, sc1 -> plain, us
// (profiles/r02r_sweep_store_policy.log): tiled slab 32 x 1.69 M f32 32.78 -> 31.87, 64 x 1.23 M
// f32 47.53 -> 46.30, 128 x 2.66 M bf16 103.65 -> 102.51, 128 x 85 354 f32 8.88 -> 8.76;
// separate buffers 128 x 2.66 M bf16 105.81 -> 103.70, 128 x 665 511 bf16 28.52 -> 28.08.
// Larger outputs lose: 64 x 4.93 M f32 (19.7 MB) 192.8 -> 203.7, 128 x 21.3 M bf16 791.4 ->
// 812.8, 8 x 25 M f32 130.4 -> 135.7; 16-peer passes (G = 16) lose at every size tried.
int vec_store_policy(int variant, int64_t out_bytes) {
  return variant == 9 && out_bytes <= (int64_t{8} << 20) ? 21 : variant;
}

constexpr int64_t kWideMaxChunks = 64 * 1024;
bool use_wide(int64_t n_chunks, int n_peers, int elems_per_chunk) {
  if (n_peers <= kGroup) return false;
  return n_chunks < kWideMaxChunks || (elems_per_chunk == 8 && n_peers > 32);
}

// The peer-major big-tile kernel (16 KiB of output per wave) where it beats the 64 x 1
// stream in interleaved A/B on MI355X (profiles/r01_ab_bigtile*.log, r01s6_ab_bigtile_*.log):
//  * fp32, 8, 16 or 32 peers, when the big tiles fill their last round of resident waves.  The
//    kernel runs one wave per SIMD (270 VGPRs), so 256 CUs x 4 = 1024 tiles are in flight;
//    a launch whose tile count ends just past a multiple of 1024 leaves most of the chip idle
//    in its last round and loses to the stream.  Measured (big tile vs stream, us):
//      8 x 25 M (5.96 rounds) 134.4 vs 137.5, 8 x 12.5 M (2.98) 66.3 vs 69.0, 8 x 4 M (0.95)
//      21.7 vs 24.3; but 8 x 21.3 M (5.08) 117.5 vs 116.9, 8 x 22.5 M (5.36) 123.0 vs 122.7,
//      8 x 26 M (6.20) 144.3 vs 142.5;
//      16 x 12.5 M (2.98) 124.5 vs 132.5, 16 x 16 M (3.81) 163.0 vs 167.5, 16 x 24.5 M (5.84)
//      247.8 vs 259.7; but 16 x 14 M (3.34) 150.3 vs 147.2, 16 x 21.3 M (5.08) 226.4 vs 224.3.
//      32 x 4.11 M (0.98) 79.8 vs 84.5, 32 x 8.2 M (1.96) 156.0 vs 172.8;
//      but below the 256 MiB Infinity Cache the stream wins: 8 x 3.4 M (0.81) 20.0 vs 17.8.
//    Rule: 8, 16 or 32 peers, >= 256 MiB of input, the last (or only) round >= 80 % full.
//    Otherwise, from one full round up, the balanced launch (variant 17) keeps the big tiles
//    for the whole rounds and spreads the rest over one round of 64-chunk segment workgroups
//    (profiles/r01s6_ab_bigtile_balanced.log, big tile / balanced / stream, us):
//      8 x 21.3 M 117.7 / 114.1 / 116.9, 8 x 26 M 143.6 / 139.4 / 142.7,
//      16 x 21.3 M 226.4 / 211.9 / 224.0, 16 x 14 M 150.5 / 139.6 / 148.0,
//      32 x 6.25 M 131.9 / 121.1 / 130.7; at a full last round it loses
//      (16 x 12.5 M 124.4 / 127.3 / 132.3) or ties (8 x 25 M 134.5 / 134.3 / 138.5).  With 7, 6, 5 or 3 fp32
//    peers the stream wins by 2-8 % (7 x 25 M 119.6 vs 116.6);
//  * fp64, 4-8 peers, >= 512 K chunks: 8 x 12.5 M 134.7 vs 162.1, 4 x 12.5 M 77.3 vs 86.4,
//    8 x 1 M 10.6 vs 13.0 (2 peers tie, 1 peer loses).  From one full round up the balanced
//    launch wins at every fp64 shape measured, full last round included (big tile / balanced /
//    stream: 8 x 10.65 M 119.6 / 116.3 / 137.5, 8 x 12.5 M 134.5 / 132.8 / 161.7,
//    4 x 10.65 M 65.9 / 64.7 / 72.9; profiles/r01s8_ab_f64_balanced.log).
constexpr int kBigTileChunks = 16;
constexpr int64_t kBigTileSlots = 256 * 4;  // MI355X: 256 CUs x 4 SIMDs x 1 big-tile wave
// 0: no big tiles; 16: big tiles; 17: big tiles for the whole rounds, the partial last round
// spread over one round of segment workgroups (the launch variants of the same names).
int bigtile_kind(int64_t n_chunks) {
  const int64_t tile = 64 * kBigTileChunks;
  const int64_t tiles = (n_chunks + tile - 1) / tile;
  const int64_t last = tiles % kBigTileSlots;
  if (tiles > 0 && (last == 0 || last * 5 >= kBigTileSlots * 4)) return 16;
  return tiles >= kBigTileSlots ? 17 : 0;
}
constexpr int64_t kMallBytes = int64_t{256} << 20;  // Infinity Cache: smaller inputs favour the stream
int use_bigtile(int64_t n_chunks, int elems_per_chunk, int n_peers) {
  if (elems_per_chunk == 4)
    return (n_peers == 8 || n_peers == 16 || n_peers == 32) && n_peers * n_chunks * 16 >= kMallBytes
               ? bigtile_kind(n_chunks)
               : 0;
  if (elems_per_chunk == 2) {  // fp64: balanced from one full round up, even when the last is full
    if (n_peers < 4 || n_peers > 8 || n_chunks < (int64_t{1} << 19)) return 0;
    return n_chunks >= kBigTileSlots * 64 * kBigTileChunks ? 17 : 16;
  }
  return 0;
}

Launch resolve(const dla_launch_cfg_t* cfg) {
  // default: nt loads + sc1 stores (+3.5 % over plain stores on every box measured)
  Launch l{4, true, 0, 0, 0};
  if (cfg) {
    if (cfg->variant) {
      l.variant = cfg->variant;
      l.auto_kernel = false;
    }
    l.block = cfg->block;
    l.chunks = cfg->chunks;
    l.grid_blocks = cfg->grid_blocks;
  }
  return l;
}

template <int DT, int KMAX, int BS, int CH, bool NT, int SP, bool ACC_IN>
hipError_t launch_stream(const PeerTable<typename Ops<DT>::w_t, KMAX>& tab, int n, int64_t n_elems,
                         void* out, hipStream_t s, int grid_blocks) {
  constexpr int E = Ops<DT>::E;
  const int64_t n_chunks = n_elems / E;
  const int64_t tile_chunks = static_cast<int64_t>(BS) * CH;
  const int64_t tiles = (n_chunks + tile_chunks - 1) / tile_chunks;
  int64_t grid = grid_blocks > 0 ? grid_blocks : tiles;
  if (grid > tiles) grid = tiles;
  if (grid > 0x7ffffffe) grid = 0x7ffffffe;
  if (n_elems > n_chunks * E) ++grid;  // + the ragged-tail workgroup
  if constexpr (DT == DLA_F16 && KMAX == 8) {
    if (n == kGroup) {
      hipLaunchKernelGGL((wsum_stream_kernel<DT, KMAX, BS, CH, NT, SP, ACC_IN, true>),
                         dim3(static_cast<unsigned>(grid)), dim3(BS), 0, s, tab, n, n_chunks, n_elems, out);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((wsum_stream_kernel<DT, KMAX, BS, CH, NT, SP, ACC_IN>), dim3(static_cast<unsigned>(grid)),
                     dim3(BS), 0, s, tab, n, n_chunks, n_elems, out);
  return hipGetLastError();
}

template <int DT, int KMAX, int BS, int CH, bool ACC_IN>
hipError_t launch_variant(const PeerTable<typename Ops<DT>::w_t, KMAX>& tab, int n, int64_t n_elems, void* out,
                          hipStream_t s, const Launch& l) {
  switch (l.variant) {
    case 1: return launch_stream<DT, KMAX, BS, CH, false, 0, ACC_IN>(tab, n, n_elems, out, s, l.grid_blocks);
    case 2: return launch_stream<DT, KMAX, BS, CH, true, 0, ACC_IN>(tab, n, n_elems, out, s, l.grid_blocks);
    default: return launch_stream<DT, KMAX, BS, CH, true, 2, ACC_IN>(tab, n, n_elems, out, s, l.grid_blocks);
  }
}

template <int DT, int KMAX, int BS, bool ACC_IN>
hipError_t launch_chunks(const PeerTable<typename Ops<DT>::w_t, KMAX>& tab, int n, int64_t n_elems, void* out,
                         hipStream_t s, const Launch& l, int chunks) {
  switch (chunks) {
    case 1: return launch_variant<DT, KMAX, BS, 1, ACC_IN>(tab, n, n_elems, out, s, l);
    case 2: return launch_variant<DT, KMAX, BS, 2, ACC_IN>(tab, n, n_elems, out, s, l);
    case 4: return launch_variant<DT, KMAX, BS, 4, ACC_IN>(tab, n, n_elems, out, s, l);
    default: return hipErrorInvalidValue;
  }
}

template <int DT, int KMAX, bool ACC_IN>
hipError_t launch_wide(const PeerTable<typename Ops<DT>::w_t, KMAX>& tab, int n, int64_t n_elems, void* out,
                       hipStream_t s) {
  // peers in flight per lane: every peer of the pass up to 64 words (f64: 32 double words)
  constexpr int kWordCap = sizeof(typename Ops<DT>::word_t) == 8 ? 32 : 64;
  constexpr int G = KMAX < kWordCap ? KMAX : kWordCap;
  const int64_t n_words = n_elems / Ops<DT>::WE;
  int64_t grid = (n_words + 63) / 64;
  if (n_elems > n_words * Ops<DT>::WE) ++grid;  // + the ragged-tail workgroup
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL((wsum_wide_kernel<DT, KMAX, G, ACC_IN>), dim3(static_cast<unsigned>(grid)), dim3(64), 0, s,
                     tab, n, n_words, n_elems, out);
  return hipGetLastError();
}

// DLA_VEC_LDS_PAD=bytes (A/B knob, default 0): dynamic LDS reserved per workgroup of the tiled vector
// kernel, which caps its workgroups per CU at 160 KiB / (bytes + its static LDS) — an occupancy
// experiment (fewer waves, fewer DRAM pages open at once), nothing reads it.
unsigned vec_lds_pad() {
  static const unsigned pad = [] {
    const char* v = tuning_env("DLA_VEC_LDS_PAD");
    const long b = v ? std::atol(v) : 0;
    return static_cast<unsigned>(b < 0 ? 0 : b > 65536 ? 65536 : b);
  }();
  return pad;
}

// Workgroups per CU the tiled vector kernel is capped at (0: uncapped), through dynamic LDS that only
// W workgroups fit.  Uncapped, the one-wave workgroups fill a CU to their register limit (32 for the
// 8-peer f32 instance); past a certain number of 512-byte loads in flight per CU more waves only keep
// more DRAM rows open at once (the counters: profiles/r03ab/pmc_summary.json — capped, the north star's
// waves spend 6 % of their life waiting instead of 46 %, on the same bytes).  The rule (round 4,
// replacing round 3's per-peer-count table): a wave's first fold round issues r1 loads of 512 B
// (r1 = G, or the largest power of two <= the pass's peers when they are fewer than G: the tail splits
// into rounds of G/2, G/4, ...), and
//     W = round(Q / r1),  Q = 112 loads (56 KiB) per CU when the pass folds in ONE round,
//                         Q = 192 loads (96 KiB) when it folds in several (its waves wait between rounds
//                         with fewer loads out, so more of them are needed for the same bytes in flight),
// applied to passes over more than the Infinity Cache (>= 256 MiB of input) whose W is below the
// kernel's own register-limited occupancy.  It reproduces the sweeps it is fitted to (profiles/r03x,
// r03y, r03ac, us): the north star 8 x 25 M f32 129.7 -> 125.8-126.3 at W = 14 (W 13: 131.0, 12: 134.9,
// 16: 127.6), 8 x 50 M bf16 130.0 -> 125.1; 4 x 25 M f32 73.6 -> 70.0 (W 26-28; rule 28); 9-15 peers x 25 M
// f32 (8 + smaller rounds, rule 24) 3.1-4.5 % faster (W 24 within 0.5 % of each count's best); 2, 3, 5, 6
// and 7 peers (rule 56, 96, 48: at or above the register limit) uncapped, where every cap measured lost.
// Exceptions, each an interleaved A/B against the rule: 12 peers (8 + 4) at W = 15, round 3's table value
// — the rule's 24 read 1.2 % and 0.85 % slower on two boxes (185.98 / 183.79 us, 185.64 / 184.08:
// profiles/r04c/cap_ab.log, profiles/r04d/cap_ab.log, spread elsewhere <= 0.35 %); 16 peers in one round of 16,
// and passes of >= 32 peers — register-limited at 16 waves per CU and holding 32 x 512 B per wave — which
// over >= 1 GiB fold 16 peers per round under W = 8 (32 x 10 M f32 199.3 -> 191.5, 64 x 4.93 M f32 192.2
// -> 184.3, 128 x 21.3 M bf16 813.8 -> 803.3, profiles/r03ai) and below it run uncapped (configs[4]'s
// 681 MB share and configs[3']'s 316 MB bucket lose with any cap).
// Round 5 lowered the floor to 160 MiB for passes of exactly 8 peers (the north star's 4-way strong-split
// bucket, 8 x 6.25 M f32 = 200 MB: W = 14 33.7-34.0 us against 34.8-34.9 uncapped; its 8-way bucket,
// 100 MB, and the 64-peer buckets tie or lose with any cap, profiles/r05p/cap.jsonl).
// In the tuning build DLA_VEC_WGS_PER_CU=W overrides the policy and DLA_VEC_CAP_TABLE=1 restores the
// round-3 table (A/B sweeps).
int vec_wgs_env() {
  static const int env = [] {
    const char* v = tuning_env("DLA_VEC_WGS_PER_CU");
    return v ? std::atoi(v) : -1;
  }();
  return env;
}

constexpr int kLoadsPerCuOneRound = 112;
constexpr int kLoadsPerCuRounds = 192;

// Round 3's measured table (tuning build only: the A/B reference of the rule).
int vec_wgs_cap_table(int n_peers, int64_t in_bytes) {
  if (n_peers >= 32) return in_bytes >= (int64_t{1} << 30) ? 8 : 0;
  switch (n_peers) {
    case 4: return 26;
    case 8: return 14;
    case 9: return 24;
    case 10: return 20;
    case 11: return 24;
    case 12: return 15;
    case 13: return 24;
    case 14: return 20;
    case 15: return 24;
    case 16: return 10;
    default: return 0;
  }
}

// n_peers: the pass's peers; G: peers per fold round of the kernel instance; natural: the workgroups
// per CU the instance reaches by its registers alone.
int vec_wgs_cap(int n_peers, int G, int64_t n_vecs, int natural) {
  const int env = vec_wgs_env();
  if (env >= 0) return env;
  const int64_t in_bytes = static_cast<int64_t>(n_peers) * n_vecs * 8;
  if (in_bytes < (n_peers == 8 ? (int64_t{160} << 20) : (int64_t{256} << 20))) return 0;
  static const bool table = [] {
    const char* v = tuning_env("DLA_VEC_CAP_TABLE");
    return v && std::atoi(v) == 1;
  }();
  if (table) return vec_wgs_cap_table(n_peers, in_bytes);
  if (n_peers >= 32) return in_bytes >= (int64_t{1} << 30) ? 8 : 0;  // exception (see above)
  if (n_peers > 16) return 0;                                        // 17-31 peers: never measured
  if (n_peers == 16 && G == 16) return 10;                           // exception (see above)
  if (n_peers == 12 && G == 16) return 15;                           // exception (see above)
  int r1 = G;
  if (n_peers < G) {
    r1 = 1;
    while (r1 * 2 <= n_peers) r1 *= 2;
  }
  const int q = n_peers == r1 ? kLoadsPerCuOneRound : kLoadsPerCuRounds;  // one fold round, or several
  const int w = (q + r1 / 2) / r1;
  return w < natural ? w : 0;
}

// Workgroups per CU a 64-thread kernel reaches without a cap (its register limit).
template <class K>
int natural_wgs_of(K kernel) {
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, 64, 0) != hipSuccess || b <= 0) {
    (void)hipGetLastError();
    return 32;
  }
  return b;
}

// Dynamic LDS per workgroup that caps a kernel whose own LDS is static_lds bytes at `wgs`
// workgroups per CU (allocations in 512-byte blocks); DLA_VEC_LDS_PAD's raw bytes when uncapped.
unsigned lds_pad_for(size_t static_lds, int wgs) {
  if (wgs <= 0) return vec_lds_pad();
  static const int64_t lds_cu = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess || v <= 0)
      v = 160 << 10;
    return static_cast<int64_t>(v);
  }();
  const int64_t per = lds_cu / wgs / 512 * 512;
  return per > static_cast<int64_t>(static_lds) ? static_cast<unsigned>(per - static_lds) : 0;
}

// The kernels over separate peer buffers (row-major wsum_vec_kernel, the many-tensor
// wsum_multi_vec_kernel) with the tiled kernel's table lose (google_speech ResNet-34 x 16 bf16
// device modules 135.3-135.8 -> 150.3-150.8 us, profiles/r03ad; 16 x 25 M f32 rows 253.6 at best
// against 250.7 for the big tile, profiles/r03ag), except 8-peer passes of the row-major kernel
// over >= 256 MiB at W = 16: 8 x 25 M f32 134.1 -> 129.4 us (and 134.7 for the big tile it now
// replaces), 8 x 50 M bf16 134.8 -> 129.0 (profiles/r03ag).  `multi`: the many-tensor kernel, kept
// uncapped (unmeasured at 8 peers).  DLA_VEC_CAP_ROWS=1 applies the whole tiled table, =0 none (A/B).
int vec_wgs_cap_rows(int dt, int n_peers, int64_t n_vecs, bool multi = false) {
  static const int env = [] {
    const char* v = tuning_env("DLA_VEC_CAP_ROWS");
    return v ? std::atoi(v) : -1;
  }();
  if (env == 1) return vec_wgs_cap_table(n_peers, static_cast<int64_t>(n_peers) * n_vecs * 8);
  if (env == 0 || multi) return 0;
  if (vec_wgs_env() >= 0) return vec_wgs_env();
  return n_peers == 8 && static_cast<int64_t>(n_peers) * n_vecs * 8 >= (int64_t{256} << 20) ? 16 : 0;
}

template <class K>
size_t static_lds_of(K kernel) {
  hipFuncAttributes a{};
  return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(kernel)) == hipSuccess ? a.sharedSizeBytes
                                                                                       : size_t{1024};
}

// Variants 9-12: the vector-per-lane kernel (VW dwords per lane, G peers in flight per lane).
template <int DT, int KMAX, bool ACC_IN>
hipError_t launch_vec(const PeerTable<typename Ops<DT>::w_t, KMAX>& tab, int n, int64_t n_elems, void* out,
                      hipStream_t s, int variant) {
  if constexpr (DT == DLA_F64) {
    return hipErrorInvalidValue;
  } else {
    constexpr int WE = Ops<DT>::WE;
#define DLA_VEC(G_, VW_, PST_)                                                                                   \
  do {                                                                                                     \
    constexpr int G = KMAX < (G_) ? KMAX : (G_);                                                           \
    const int64_t n_vecs = n_elems / ((VW_) * WE);                                                         \
    int64_t grid = (n_vecs + 63) / 64;                                                                     \
    if (n_elems > n_vecs * (VW_) * WE) ++grid;                                                             \
    if (grid < 1 || grid > 0x7fffffff) return hipErrorInvalidValue;                                        \
    static const size_t st_lds = static_lds_of(&wsum_vec_kernel<DT, KMAX, G, VW_, ACC_IN, false, PST_>);    \
    const unsigned lds_pad = lds_pad_for(st_lds, vec_wgs_cap_rows(DT, n, n_vecs));                         \
    hipLaunchKernelGGL((wsum_vec_kernel<DT, KMAX, G, VW_, ACC_IN, false, PST_>), dim3(static_cast<unsigned>(grid)), dim3(64), \
                       lds_pad, s, tab, n, n_vecs, n_elems, out);                                          \
  } while (0)
    switch (variant) {
      case 9: DLA_VEC(32, 2, false); break;
      case 21: DLA_VEC(32, 2, true); break;
      default: DLA_VEC(16, 2, false); break;  // 12
    }
#undef DLA_VEC
    return hipGetLastError();
  }
}

// The tile-interleaved slab (dla_wsum_slab_tiled) through the vector-per-lane kernel: variant 8 =
// dwordx2 x 8 peers in flight (28: with plain stores), 12 = dwordx2 x 16, 21 = dwordx2 x 32 with plain
// stores, otherwise (default, 9) dwordx2 x 32.
template <int DT, int KMAX, bool ACC_IN>
hipError_t launch_vec_tiled(const PeerTable<typename Ops<DT>::w_t, KMAX>& tab, int n, int64_t n_elems, void* out,
                            hipStream_t s, int variant, int tshift_e, int64_t tstride_e) {
  if constexpr (DT == DLA_F64) {
    return hipErrorInvalidValue;
  } else {
    constexpr int WE = Ops<DT>::WE;
#define DLA_VECT(G_, VW_, PST_)                                                                                     \
  do {                                                                                                        \
    constexpr int G = KMAX < (G_) ? KMAX : (G_);                                                              \
    constexpr int per_vec = (VW_) * WE;                                                                       \
    int vs = 0;                                                                                               \
    while ((1 << vs) < per_vec) ++vs;                                                                         \
    if (tshift_e < vs) return hipErrorInvalidValue;                                                           \
    const int64_t n_vecs = n_elems / per_vec;                                                                 \
    int64_t grid = (n_vecs + 63) / 64;                                                                        \
    if (n_elems > n_vecs * per_vec) ++grid;                                                                   \
    if (grid < 1 || grid > 0x7fffffff) return hipErrorInvalidValue;                                           \
    static const size_t st_lds = static_lds_of(&wsum_vec_kernel<DT, KMAX, G, VW_, ACC_IN, true, PST_>);     \
    static const int natural = natural_wgs_of(wsum_vec_kernel<DT, KMAX, G, VW_, ACC_IN, true, PST_>);        \
    const unsigned lds_pad = lds_pad_for(st_lds, vec_wgs_cap(n, G, n_vecs, natural));                         \
    hipLaunchKernelGGL((wsum_vec_kernel<DT, KMAX, G, VW_, ACC_IN, true, PST_>), dim3(static_cast<unsigned>(grid)),   \
                       dim3(64), lds_pad, s, tab, n, n_vecs, n_elems, out, tshift_e - vs, tstride_e / per_vec,    \
                       tshift_e, tstride_e);                                                                  \
  } while (0)
    switch (variant) {
      case 8: DLA_VECT(8, 2, false); break;
      case 12: DLA_VECT(16, 2, false); break;
      case 21: DLA_VECT(32, 2, true); break;
      case 28: DLA_VECT(8, 2, true); break;
      default: DLA_VECT(32, 2, false); break;
    }
#undef DLA_VECT
    return hipGetLastError();
  }
}

template <int DT>
hipError_t run_tiled(const void* base, int64_t tile_elems, int tshift, int64_t stride_elems, const double* weights,
                     int n, int64_t n_elems, void* out, hipStream_t s, int variant) {
  constexpr int es = sizeof(typename Ops<DT>::elem_t);
  for (int k0 = 0; k0 < n; k0 += kMaxPeersPerPass) {
    const int m = n - k0 < kMaxPeersPerPass ? n - k0 : kMaxPeersPerPass;
    hipError_t e;
#define DLA_TILED_PASS(KM)                                                                                   \
  do {                                                                                                       \
    PeerTable<typename Ops<DT>::w_t, KM> tab;                                                                \
    std::memset(&tab, 0, sizeof(tab));                                                                       \
    for (int k = 0; k < m; ++k) {                                                                            \
      tab.p[k] = static_cast<const char*>(base) + (k0 + k) * tile_elems * es;                                \
      tab.w[k] = static_cast<typename Ops<DT>::w_t>(weights[k0 + k]);                                        \
    }                                                                                                        \
    e = k0 > 0 ? launch_vec_tiled<DT, KM, true>(tab, m, n_elems, out, s, variant, tshift, stride_elems)       \
               : launch_vec_tiled<DT, KM, false>(tab, m, n_elems, out, s, variant, tshift, stride_elems);     \
  } while (0)
    if (m <= 8)
      DLA_TILED_PASS(8);
    else if (m <= 32)
      DLA_TILED_PASS(32);
    else
      DLA_TILED_PASS(kMaxPeersPerPass);
#undef DLA_TILED_PASS
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <int DT, int KMAX>
hipError_t launch_bigtile(const PeerTable<typename Ops<DT>::w_t, KMAX>& tab, int n, int64_t n_elems, void* out,
                          hipStream_t s, bool balanced) {
  constexpr int BT = kBigTileChunks;
  constexpr int64_t kTile = 64 * BT;
  const int64_t n_chunks = n_elems / Ops<DT>::E;
  const int64_t n_full = n_chunks / kTile;
  int64_t n_big = n_full, n_seg_wg = n_full * kTile < n_chunks ? 1 : 0;  // + the partial-tile workgroup
  if (balanced) {
    n_big = n_full / kBigTileSlots * kBigTileSlots;
    const int64_t segs = (n_chunks - n_big * kTile + 63) / 64;
    n_seg_wg = segs < kBigTileSlots ? segs : kBigTileSlots;
  }
  int64_t grid = n_big + n_seg_wg;
  if (n_elems > n_chunks * Ops<DT>::E) ++grid;  // + the ragged-tail workgroup
  if (grid < 1 || grid > 0x7fffffff) return hipErrorInvalidValue;
  const dim3 g(static_cast<unsigned>(grid)), b(64);
#define DLA_BIGTILE(NPV)                                                                                      \
  hipLaunchKernelGGL((wsum_bigtile_kernel<DT, NPV, BT, KMAX>), g, b, 0, s, tab, n_chunks, n_elems, n_big, n_seg_wg, \
                     out)
  if constexpr (KMAX == 32) {  // 16 or 32 fp32 peers
    switch (n) {
      case 16: DLA_BIGTILE(16); break;
      case 32: DLA_BIGTILE(32); break;
      default: return hipErrorInvalidValue;
    }
  } else {
    switch (n) {
      case 1: DLA_BIGTILE(1); break;
      case 2: DLA_BIGTILE(2); break;
      case 3: DLA_BIGTILE(3); break;
      case 4: DLA_BIGTILE(4); break;
      case 5: DLA_BIGTILE(5); break;
      case 6: DLA_BIGTILE(6); break;
      case 7: DLA_BIGTILE(7); break;
      case 8: DLA_BIGTILE(8); break;
      default: return hipErrorInvalidValue;
    }
  }
#undef DLA_BIGTILE
  return hipGetLastError();
}

template <int DT, int KMAX, bool ACC_IN>
hipError_t launch_pass(const PeerTable<typename Ops<DT>::w_t, KMAX>& tab, int n, int64_t n_elems,
                       void* out, hipStream_t s, const Launch& l, bool aligned) {
  if (!aligned) {
    int64_t blocks = (n_elems + kBlock - 1) / kBlock;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL((wsum_scalar_kernel<DT, KMAX, ACC_IN>), dim3(static_cast<unsigned>(blocks)),
                       dim3(kBlock), 0, s, tab, n, n_elems, out);
    return hipGetLastError();
  }
  if (l.variant == 9 || l.variant == 12 || l.variant == 21) {
    if constexpr (DT != DLA_F64) return launch_vec<DT, KMAX, ACC_IN>(tab, n, n_elems, out, s, l.variant);
  }
  if constexpr ((DT == DLA_BF16 || DT == DLA_F16) && KMAX == 8) {
    // up to 8 bf16 / f16 peers: the vector-per-lane kernel too (r02 A/B against the 16-byte
    // stream, profiles/r02w_vec8.log, us: 6 x 25 M bf16 51.9 vs 58.8, 8 x 50 M bf16 136.3 vs
    // 138.5, 4 x 50 M f16 72.4 vs 73.1; fp32 keeps the stream / big tile: 4 x 25 M 73.2 vs 72.3,
    // 8 x 25 M 134.9 vs 135.1)
    if (l.auto_kernel) return launch_vec<DT, KMAX, ACC_IN>(tab, n, n_elems, out, s, vec_variant(n));
  }
  if constexpr (DT != DLA_F64 && KMAX != 8) {
    // more than 8 peers: the vector-per-lane kernel, unless an fp32 big tile applies (below)
    const bool big = DT == DLA_F32 && !ACC_IN && (n == 16 || n == 32) &&
                     use_bigtile(n_elems / Ops<DT>::E, Ops<DT>::E, n) != 0;
    if (l.auto_kernel && !big)
      return launch_vec<DT, KMAX, ACC_IN>(tab, n, n_elems, out, s,
                                          vec_store_policy(vec_variant(n), n_elems * int64_t{sizeof(typename Ops<DT>::elem_t)}));
  }
  if (l.variant == 8 || (l.auto_kernel && use_wide(n_elems / Ops<DT>::E, n, Ops<DT>::E)))
    return launch_wide<DT, KMAX, ACC_IN>(tab, n, n_elems, out, s);
  if constexpr (KMAX == 8 && DT == DLA_F32) {
    // 8 fp32 peers over >= 256 MiB: the row-major vector kernel at 16 workgroups per CU beats the
    // big tile (8 x 25 M: 129.4 vs 134.7 us, profiles/r03ag)
    if (l.auto_kernel && n == 8 && int64_t{n} * n_elems * 4 >= kMallBytes)
      return launch_vec<DT, KMAX, ACC_IN>(tab, n, n_elems, out, s, vec_variant(n));
  }
  if constexpr (KMAX == 8 && !ACC_IN && (DT == DLA_F32 || DT == DLA_F64)) {
    const int kind = l.auto_kernel ? use_bigtile(n_elems / Ops<DT>::E, Ops<DT>::E, n) : l.variant;
    if (kind == 16 || kind == 17) return launch_bigtile<DT, KMAX>(tab, n, n_elems, out, s, kind == 17);
  }
  if constexpr (KMAX == 32 && !ACC_IN && DT == DLA_F32) {
    // instantiated for exactly 16 and 32 peers; any other count of a forced 16/17 takes the stream
    const int kind = l.auto_kernel ? use_bigtile(n_elems / Ops<DT>::E, Ops<DT>::E, n) : l.variant;
    if ((kind == 16 || kind == 17) && (n == 16 || n == 32))
      return launch_bigtile<DT, KMAX>(tab, n, n_elems, out, s, kind == 17);
  }
  int block = l.block, chunks = l.chunks;
  if (!block || !chunks) {
    int b, c;
    shape_for(n_elems / Ops<DT>::E, n, Ops<DT>::E, &b, &c);
    if (!block) block = b;
    if (!chunks) chunks = c;
  }
  if (block == 64) return launch_chunks<DT, KMAX, 64, ACC_IN>(tab, n, n_elems, out, s, l, chunks);
  return launch_chunks<DT, KMAX, 256, ACC_IN>(tab, n, n_elems, out, s, l, chunks);
}

template <int DT, int KMAX>
hipError_t run_pass(const void* const* peers, const double* weights, int n, int64_t n_elems,
                    void* out, hipStream_t s, const Launch& l, bool acc_in) {
  using W = typename Ops<DT>::w_t;
  PeerTable<W, KMAX> tab;
  std::memset(&tab, 0, sizeof(tab));
  bool aligned = (reinterpret_cast<uintptr_t>(out) & 15u) == 0;
  for (int k = 0; k < n; ++k) {
    tab.p[k] = peers[k];
    tab.w[k] = static_cast<W>(weights[k]);  // RNE double -> op-math (fedavg.py:25 `w * p1`)
    aligned = aligned && (reinterpret_cast<uintptr_t>(peers[k]) & 15u) == 0;
  }
  return acc_in ? launch_pass<DT, KMAX, true>(tab, n, n_elems, out, s, l, aligned)
                : launch_pass<DT, KMAX, false>(tab, n, n_elems, out, s, l, aligned);
}

template <int DT>
hipError_t run(const void* const* peers, const double* weights, int n, int64_t n_elems, void* out,
               hipStream_t s, const Launch& l, bool acc_in = false) {
  // Passes of at most kMaxPeersPerPass peers; pass j > 0 folds its peers into
  // the running sum held in `out`, so the list order is kept exactly (acc_in: so does pass 0 —
  // `out` already holds the fold of earlier peers).
  for (int k0 = 0; k0 < n; k0 += kMaxPeersPerPass) {
    const int m = n - k0 < kMaxPeersPerPass ? n - k0 : kMaxPeersPerPass;
    const bool acc = acc_in || k0 > 0;
    hipError_t e;
    if (m <= 8)
      e = run_pass<DT, 8>(peers + k0, weights + k0, m, n_elems, out, s, l, acc);
    else if (m <= 32)
      e = run_pass<DT, 32>(peers + k0, weights + k0, m, n_elems, out, s, l, acc);
    else
      e = run_pass<DT, kMaxPeersPerPass>(peers + k0, weights + k0, m, n_elems, out, s, l, acc);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Batches of up to MAXSEG tensors per launch (see wsum_multi_kernel).
template <int DT, int NP, int MAXSEG>
hipError_t launch_multi(const int* tensors, int count, const void* const* peer_ptrs, void* const* outs,
                        const int64_t* numels, const double* weights, int n, hipStream_t s) {
  using W = typename Ops<DT>::w_t;
  SegTable<W, NP, MAXSEG> tab;
  std::memset(&tab, 0, sizeof(tab));
  for (int k = 0; k < n; ++k) tab.w[k] = static_cast<W>(weights[k]);
  int64_t cum = 0;
  for (int i = 0; i < count; ++i) {
    const int t = tensors[i];
    for (int k = 0; k < n; ++k) tab.p[i][k] = peer_ptrs[static_cast<int64_t>(t) * n + k];
    tab.out[i] = outs[t];
    tab.n_elems[i] = numels[t];
    const int64_t chunks = numels[t] / Ops<DT>::E;
    const int64_t tiles = chunks ? (chunks + kBlock - 1) / kBlock : 1;
    cum += tiles;
    tab.tile_end[i] = cum;
  }
  hipLaunchKernelGGL((wsum_multi_kernel<DT, NP, MAXSEG, 2>), dim3(static_cast<unsigned>(cum)), dim3(kBlock), 0, s,
                     tab, count, n);
  return hipGetLastError();
}

template <int DT, int NP, int MAXSEG>
hipError_t run_multi(const std::vector<int>& packed, const void* const* peer_ptrs, void* const* outs,
                     const int64_t* numels, const double* weights, int n, hipStream_t s) {
  for (size_t i = 0; i < packed.size(); i += MAXSEG) {
    const int count = static_cast<int>(packed.size() - i < MAXSEG ? packed.size() - i : MAXSEG);
    hipError_t e = launch_multi<DT, NP, MAXSEG>(packed.data() + i, count, peer_ptrs, outs, numels, weights, n, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <int DT>
hipError_t run_multi_dt(const std::vector<int>& packed, const void* const* peer_ptrs, void* const* outs,
                        const int64_t* numels, const double* weights, int n, hipStream_t s) {
  if (n <= 8) return run_multi<DT, 8, 32>(packed, peer_ptrs, outs, numels, weights, n, s);
  return run_multi<DT, 32, 8>(packed, peer_ptrs, outs, numels, weights, n, s);
}

// dla_wsum_multi_table: the device table is, per launch of up to 256 tensors, [MultiIndex][MultiSeg x mc]
// (16-byte aligned), then the m x n_peers peer pointers of every tensor.
int64_t multi_chunk_bytes(int mc) {
  return static_cast<int64_t>(sizeof(MultiIndex)) + (static_cast<int64_t>(mc) * sizeof(MultiSeg) + 15) / 16 * 16;
}

int64_t multi_table_bytes(int n_tensors, int n_peers) {
  int64_t b = 0;
  for (int c0 = 0; c0 < n_tensors; c0 += kMultiTensorsPerLaunch)
    b += multi_chunk_bytes(n_tensors - c0 < kMultiTensorsPerLaunch ? n_tensors - c0 : kMultiTensorsPerLaunch);
  return b + static_cast<int64_t>(n_tensors) * n_peers * 8;
}

template <int DT, int KMAX, int G, bool ACC_IN>
hipError_t launch_multi_vec(const MultiIndex* idx, const MultiSeg* segs, int n_seg, int64_t grid, int k0, int pm,
                            const double* weights, bool plain, hipStream_t s) {
  using W = typename Ops<DT>::w_t;
  WeightTable<W, KMAX> wt;
  std::memset(&wt, 0, sizeof(wt));
  for (int k = 0; k < pm; ++k) wt.w[k] = static_cast<W>(weights[k0 + k]);  // RNE double -> op-math
  const dim3 g(static_cast<unsigned>(grid)), bl(64);
  const int wgs = vec_wgs_cap_rows(DT, pm, grid * 64, true);  // every workgroup folds 64 vectors
  if (plain) {
    static const size_t st_lds = static_lds_of(&wsum_multi_vec_kernel<DT, KMAX, G, ACC_IN, true>);
    hipLaunchKernelGGL((wsum_multi_vec_kernel<DT, KMAX, G, ACC_IN, true>), g, bl, lds_pad_for(st_lds, wgs), s, idx,
                       segs, n_seg, k0, pm, wt);
  } else {
    static const size_t st_lds = static_lds_of(&wsum_multi_vec_kernel<DT, KMAX, G, ACC_IN, false>);
    hipLaunchKernelGGL((wsum_multi_vec_kernel<DT, KMAX, G, ACC_IN, false>), g, bl, lds_pad_for(st_lds, wgs), s, idx,
                       segs, n_seg, k0, pm, wt);
  }
  return hipGetLastError();
}

template <int DT, bool ACC_IN>
hipError_t launch_multi_vec_pass(const MultiIndex* idx, const MultiSeg* segs, int n_seg, int64_t grid, int k0, int pm,
                                 const double* weights, bool plain, hipStream_t s) {
  // peers in flight per lane as the single-tensor vec kernel (vec_variant): 32 for passes of >= 32
  // peers, 16 above 8, else 8
  if (pm > 32)
    return launch_multi_vec<DT, kMaxPeersPerPass, 32, ACC_IN>(idx, segs, n_seg, grid, k0, pm, weights, plain, s);
  if (pm == 32) return launch_multi_vec<DT, 32, 32, ACC_IN>(idx, segs, n_seg, grid, k0, pm, weights, plain, s);
  if (pm > 8) return launch_multi_vec<DT, 32, 16, ACC_IN>(idx, segs, n_seg, grid, k0, pm, weights, plain, s);
  return launch_multi_vec<DT, 8, 8, ACC_IN>(idx, segs, n_seg, grid, k0, pm, weights, plain, s);
}

// The table's host -> device copy (defined with the library's stream / event state below); `moved` is
// the call's algorithmic bytes (its kernels' duration scale).
hipError_t upload_table(char* td, const char* th, size_t bytes, int64_t moved, hipStream_t s);

template <int DT>
hipError_t run_multi_table(const std::vector<int>& packed, const void* const* peer_ptrs, void* const* outs,
                           const int64_t* numels, const double* weights, int n, char* th, char* td, hipStream_t s,
                           bool acc_in) {
  constexpr int per_vec = 2 * Ops<DT>::WE;  // elements per 8-byte vector
  const int m = static_cast<int>(packed.size());
  const int64_t ptab_off = multi_table_bytes(m, n) - static_cast<int64_t>(m) * n * 8;
  const void** ptab = reinterpret_cast<const void**>(th + ptab_off);
  int64_t out_bytes = 0;
  for (int i = 0; i < m; ++i) out_bytes += numels[packed[i]] * static_cast<int64_t>(sizeof(typename Ops<DT>::elem_t));
  // plain output stores for passes of >= 32 peers writing <= 8 MiB in all (vec_store_policy)
  const bool plain_ok = out_bytes <= (int64_t{8} << 20);
  struct Launch1 { int64_t off; int mc; int64_t grid; };
  std::vector<Launch1> launches;
  int64_t off = 0;
  for (int c0 = 0; c0 < m; c0 += kMultiTensorsPerLaunch) {
    const int mc = m - c0 < kMultiTensorsPerLaunch ? m - c0 : kMultiTensorsPerLaunch;
    MultiIndex* ix = reinterpret_cast<MultiIndex*>(th + off);
    MultiSeg* segs = reinterpret_cast<MultiSeg*>(th + off + sizeof(MultiIndex));
    for (int q = 0; q < 256; ++q) ix->fine[q] = 0x7fffffff;
    int64_t wg = 0;
    for (int i = 0; i < mc; ++i) {
      const int t = packed[c0 + i];
      const int64_t nv = numels[t] / per_vec;
      segs[i].wg_begin = wg;
      segs[i].n_vecs = nv;
      segs[i].n_elems = numels[t];
      segs[i].out = outs[t];
      segs[i].ptrs = reinterpret_cast<const void* const*>(td + ptab_off + static_cast<int64_t>(c0 + i) * n * 8);
      std::memcpy(ptab + static_cast<int64_t>(c0 + i) * n, peer_ptrs + static_cast<int64_t>(t) * n, sizeof(void*) * n);
      ix->fine[i] = static_cast<int32_t>(wg);
      wg += (nv + 63) / 64 + (numels[t] > nv * per_vec ? 1 : 0);
      if (wg > 0x7fffffff) return hipErrorInvalidValue;
    }
    for (int q = 0; q < 16; ++q) ix->coarse[q] = ix->fine[16 * q];
    launches.push_back({off, mc, wg});
    off += multi_chunk_bytes(mc);
  }
  const int64_t moved = (static_cast<int64_t>(n) + 1) * out_bytes;
  hipError_t e = upload_table(td, th, static_cast<size_t>(multi_table_bytes(m, n)), moved, s);
  if (e != hipSuccess) return e;
  for (int k0 = 0; k0 < n; k0 += kMaxPeersPerPass) {
    const int pm = n - k0 < kMaxPeersPerPass ? n - k0 : kMaxPeersPerPass;
    for (const Launch1& L : launches) {
      const MultiIndex* ix = reinterpret_cast<const MultiIndex*>(td + L.off);
      const MultiSeg* segs = reinterpret_cast<const MultiSeg*>(td + L.off + sizeof(MultiIndex));
      e = k0 > 0 || acc_in
              ? launch_multi_vec_pass<DT, true>(ix, segs, L.mc, L.grid, k0, pm, weights, plain_ok && pm >= 32, s)
              : launch_multi_vec_pass<DT, false>(ix, segs, L.mc, L.grid, k0, pm, weights, plain_ok && pm >= 32, s);
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

template <int DT, int KMAX>
hipError_t mean_pass(const void* const* peers, int n, int n_total, int64_t n_elems, void* out, hipStream_t s,
                     bool acc_in, bool divide) {
  using W = typename Ops<DT>::w_t;
  PeerTable<W, KMAX> tab;
  std::memset(&tab, 0, sizeof(tab));
  bool aligned = (reinterpret_cast<uintptr_t>(out) & 15u) == 0;
  for (int k = 0; k < n; ++k) {
    tab.p[k] = peers[k];
    tab.w[k] = W(1);
    aligned = aligned && (reinterpret_cast<uintptr_t>(peers[k]) & 15u) == 0;
  }
  constexpr int E = Ops<DT>::E;
  const int64_t n_chunks = aligned ? n_elems / E : 0;
  int64_t grid = aligned ? (n_chunks + 63) / 64 : (n_elems + 63) / 64;
  if (!aligned && grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  const typename Ops<DT>::acc_t d = static_cast<typename Ops<DT>::acc_t>(n_total);
#define DLA_MEAN_L(AI, AL)                                                                                  \
  hipLaunchKernelGGL((mean_kernel<DT, KMAX, AI, AL>), dim3(static_cast<unsigned>(grid)), dim3(64), 0, s, tab, n, \
                     n_chunks, n_elems, out, d, divide ? 1 : 0)
  if (acc_in) {
    if (aligned) DLA_MEAN_L(true, true); else DLA_MEAN_L(true, false);
  } else {
    if (aligned) DLA_MEAN_L(false, true); else DLA_MEAN_L(false, false);
  }
#undef DLA_MEAN_L
  return hipGetLastError();
}

template <int DT>
hipError_t run_mean(const void* const* peers, int n, int64_t n_elems, void* out, hipStream_t s) {
  for (int k0 = 0; k0 < n; k0 += kMaxPeersPerPass) {
    const int m = n - k0 < kMaxPeersPerPass ? n - k0 : kMaxPeersPerPass;
    const bool last = k0 + m >= n;
    hipError_t e = m <= 8 ? mean_pass<DT, 8>(peers + k0, m, n, n_elems, out, s, k0 > 0, last)
                 : m <= 32 ? mean_pass<DT, 32>(peers + k0, m, n, n_elems, out, s, k0 > 0, last)
                           : mean_pass<DT, kMaxPeersPerPass>(peers + k0, m, n, n_elems, out, s, k0 > 0, last);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

int elem_size(int dtype) {
  switch (dtype) {
    case DLA_F32: return 4;
    case DLA_BF16: return 2;
    case DLA_F16: return 2;
    case DLA_F64: return 8;
    default: return 0;
  }
}

hipError_t run_mixed(int out_dtype, const int* peer_dtypes, const void* const* peers, const double* weights, int n,
                     int64_t n_elems, void* out, hipStream_t s) {
  int64_t grid = (n_elems + kBlock - 1) / kBlock;
  if (grid > 4096) grid = 4096;  // grid-stride beyond 16 workgroups per CU
  for (int k0 = 0; k0 < n; k0 += kMaxPeersPerPass) {
    const int m = n - k0 < kMaxPeersPerPass ? n - k0 : kMaxPeersPerPass;
    MixedTable tab;
    std::memset(&tab, 0, sizeof(tab));
    for (int k = 0; k < m; ++k) {
      tab.p[k] = peers[k0 + k];
      tab.w[k] = weights[k0 + k];
      tab.dt[k] = static_cast<int8_t>(peer_dtypes[k0 + k]);
    }
    if (k0 == 0)
      hipLaunchKernelGGL(wsum_mixed_kernel<false>, dim3(static_cast<unsigned>(grid)), dim3(kBlock), 0, s, tab, m,
                         out_dtype, n_elems, out);
    else
      hipLaunchKernelGGL(wsum_mixed_kernel<true>, dim3(static_cast<unsigned>(grid)), dim3(kBlock), 0, s, tab, m,
                         out_dtype, n_elems, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

int wsum_impl(int dtype, const void* const* peers, const double* weights, int n_peers,
              int64_t n_elems, void* out, void* stream, const dla_launch_cfg_t* cfg, bool acc_in = false) {
  g_last_error.clear();
  if (elem_size(dtype) == 0) return fail(DLA_E_INVALID, "dla_wsum: unknown dtype " + std::to_string(dtype));
  if (n_peers < 1) return fail(DLA_E_INVALID, "dla_wsum: n_peers must be >= 1 (fedavg.py:20 indexes models[0])");
  if (n_elems < 0) return fail(DLA_E_INVALID, "dla_wsum: n_elems < 0");
  if (!peers || !weights) return fail(DLA_E_INVALID, "dla_wsum: null peers/weights array");
  if (n_elems == 0) return DLA_OK;
  if (!out) return fail(DLA_E_INVALID, "dla_wsum: null out");
  for (int k = 0; k < n_peers; ++k)
    if (!peers[k]) return fail(DLA_E_INVALID, "dla_wsum: null peer pointer " + std::to_string(k));
  if (acc_in) {  // out carries the running sum from the start: it may alias no peer
    for (int k = 0; k < n_peers; ++k)
      if (peers[k] == out) return fail(DLA_E_ALIAS, "dla_wsum: out aliases peer " + std::to_string(k) + " (acc_in)");
  } else if (n_peers > kMaxPeersPerPass) {
    // Multi-pass reduce: out carries the running sum, so it may alias only peers[0].
    for (int k = 1; k < n_peers; ++k)
      if (peers[k] == out)
        return fail(DLA_E_ALIAS, "dla_wsum: out aliases peer " + std::to_string(k) +
                                     "; only peers[0] may alias out when n_peers > " +
                                     std::to_string(kMaxPeersPerPass));
  }
  const Launch l = resolve(cfg);
  if (l.variant != 1 && l.variant != 2 && l.variant != 4 && l.variant != 8 && l.variant != 9 && l.variant != 12 && l.variant != 16 &&
      l.variant != 17 && l.variant != 21)
    return fail(DLA_E_CONFIG,
                "dla_wsum: unsupported variant " + std::to_string(l.variant) + " (1, 2, 4, 8, 9, 12, 16, 17 or 21)");
  if (l.chunks != 0 && l.chunks != 1 && l.chunks != 2 && l.chunks != 4)
    return fail(DLA_E_CONFIG, "dla_wsum: chunks must be 0 (auto), 1, 2 or 4");
  if (l.block != 0 && l.block != 64 && l.block != 256)
    return fail(DLA_E_CONFIG, "dla_wsum: block must be 0 (auto), 64 or 256");
  if (l.grid_blocks < 0) return fail(DLA_E_CONFIG, "dla_wsum: grid_blocks < 0");
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e;
  switch (dtype) {
    case DLA_F32: e = run<DLA_F32>(peers, weights, n_peers, n_elems, out, s, l, acc_in); break;
    case DLA_BF16: e = run<DLA_BF16>(peers, weights, n_peers, n_elems, out, s, l, acc_in); break;
    case DLA_F16: e = run<DLA_F16>(peers, weights, n_peers, n_elems, out, s, l, acc_in); break;
    default: e = run<DLA_F64>(peers, weights, n_peers, n_elems, out, s, l, acc_in); break;
  }
  if (e != hipSuccess) return fail(static_cast<int>(e), std::string("dla_wsum: ") + hipGetErrorString(e));
  return DLA_OK;
}

// ------------------------------------------------ bucket-sharded reduce over the GPUs of one process
// the flat parameter vector splits into contiguous 256-B-aligned buckets, one per
// shard; shard s reduces its bucket of EVERY peer on its own GPU (peers on other GPUs are read
// over xGMI peer-to-peer), so every element keeps its list-order fold and the result is
// bit-identical to the one-GPU reduce.  Process-wide state (the only state the library keeps):
// the peer-access pairs it enabled and a pool of synchronisation events, both released by
// dla_shutdown().
std::mutex g_shard_mu;
std::set<std::pair<int, int>> g_peer_enabled;  // (accessing device, owning device) pairs enabled here
std::vector<std::pair<int, hipEvent_t>> g_event_pool;  // (device, event) not in use

int64_t shard_bucket_elems(int es, int64_t n_elems, int n_shards) {
  const int64_t align = 256 / es;
  int64_t per = (n_elems + n_shards - 1) / n_shards;
  return (per + align - 1) / align * align;
}

class DeviceGuard {
 public:
  DeviceGuard() { ok_ = hipGetDevice(&prev_) == hipSuccess; }
  ~DeviceGuard() {
    if (ok_) (void)hipSetDevice(prev_);
  }

 private:
  int prev_ = 0;
  bool ok_ = false;
};

// Device that owns a device pointer (-1 if it is not device memory).
int owner_device(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  if (a.type != hipMemoryTypeDevice) return -1;
  return a.device;
}

bool is_pinned_host_ptr(const void* p) {
  hipPointerAttribute_t a;
  const bool ok = hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost;
  if (!ok) (void)hipGetLastError();
  return ok;
}

bool is_device_ptr(const void* p) {
  hipPointerAttribute_t a;
  const bool ok = hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeDevice;
  if (!ok) (void)hipGetLastError();
  return ok;
}

// Page-locked host memory mapped into the device address space at the same address (hipHostMalloc,
// torch pin_memory): a kernel can read / write it across PCIe through the host pointer itself.  Only
// memory the runtime associates with the CURRENT device counts: a kernel on another GPU of the node
// reading a buffer mapped for device 0 is not something this library assumes (the host path over several
// GPUs then keeps its staging DMAs on those GPUs, which any page-locked memory serves).
bool is_mapped_host_ptr(const void* p) {
  hipPointerAttribute_t a;
  int cur = -1;
  const bool ok = hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost &&
                  a.devicePointer == p && hipGetDevice(&cur) == hipSuccess && a.device == cur;
  if (!ok) (void)hipGetLastError();
  return ok;
}

std::atomic<int64_t> g_host_in_place{0};  // host rounds whose peers the kernel read in place (dla_host_in_place_rounds)

// Peers whose flat parameter vectors are page-locked ROWS (a model decoded into a
// page-locked ingress buffer, DeviceModelManager's EVA gather, holds its tensors back to back in one
// pinned row): true when, for every peer k, every non-empty tensor t sits at row_k + start[t] bytes,
// row_k + begin is 16-byte aligned, and the row's bytes [begin, end) are page-locked and device-mapped.
// rows[k] then holds row_k (the address of flat element 0).  The host path lets the kernel read such
// rows across PCIe where they are — no pack into staging, no staging DMA (the kernel's own PCIe reads
// run at the DMA rate on this link, 53.9-54.8 GB/s).  The first peer that does not
// qualify ends the check (the reference's pageable peers cost one pointer query).
bool mapped_peer_rows(int es, int n_peers, int n_tensors, const void* const* tensors, const int64_t* start,
                      int64_t begin, int64_t end, std::vector<const char*>& rows) {
  rows.assign(n_peers, nullptr);
  for (int k = 0; k < n_peers; ++k) {
    const char* base = nullptr;
    for (int t = 0; t < n_tensors; ++t) {
      if (start[t + 1] == start[t]) continue;
      const char* b = static_cast<const char*>(tensors[static_cast<size_t>(k) * n_tensors + t]) - start[t] * es;
      if (!base) {
        base = b;
      } else if (b != base) {
        return false;
      }
    }
    if (!base || (reinterpret_cast<uintptr_t>(base + begin * es) & 15u)) return false;
    if (!is_mapped_host_ptr(base + begin * es) || !is_mapped_host_ptr(base + end * es - 1)) return false;
    rows[k] = base;
  }
  return true;
}

// Let `dev` read / write memory owned by `owner` (caller holds g_shard_mu; device set to dev).
hipError_t ensure_peer_access(int dev, int owner) {
  if (dev == owner || owner < 0 || g_peer_enabled.count({dev, owner})) return hipSuccess;
  int can = 0;
  hipError_t e = hipDeviceCanAccessPeer(&can, dev, owner);
  if (e != hipSuccess) return e;
  if (!can) return hipErrorPeerAccessUnsupported;
  e = hipDeviceEnablePeerAccess(owner, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
    return hipSuccess;  // enabled by someone else (e.g. torch): not ours to disable
  }
  if (e == hipSuccess) g_peer_enabled.insert({dev, owner});
  return e;
}

hipError_t take_event(int dev, hipEvent_t* ev) {  // caller holds g_shard_mu; device set to dev
  for (size_t i = 0; i < g_event_pool.size(); ++i) {
    if (g_event_pool[i].first == dev) {
      *ev = g_event_pool[i].second;
      g_event_pool.erase(g_event_pool.begin() + static_cast<std::ptrdiff_t>(i));
      return hipSuccess;
    }
  }
  return hipEventCreateWithFlags(ev, hipEventDisableTiming);
}

// The multi-tensor table's upload.  A copy-engine job between two kernels of the reduce's stream costs
// ~24 us of idle GPU per call (kernel end -> DMA start 9 us, the 19.6 KB DMA 6 us, DMA end -> next kernel
// 8 us: profiles/r05c, 16 google_speech ResNet-34 models, back to back), against ~6 us between two
// kernels.  Policy (profiles/r05d, modes A/B'd under DLA_TABLE_COPY in the tuning build):
//  * the stream is still busy with this library's earlier table reduces (stream_busy_through) and the
//    call moves >= 256 MiB (its kernel runs >= ~40 us: rounds back to back): the copy runs on a library
//    side stream of the device WHILE the queued kernel runs, and the calling thread waits for it
//    (~15-20 us) before enqueuing the reduce — nothing sits between the kernels (mode 3: 1.8 us from one
//    kernel's end to the next one's start, as with no upload at all; a barrier packet waiting on the
//    copy's event, mode 2, still costs ~11 us);
//  * otherwise (an idle GPU, or short kernels the host wait would outlast): a copy kernel on the stream
//    reads the page-locked table across PCIe (mode 1: 3-4 us, no copy-engine hand-off);
//  * a table that is not device-mapped page-locked memory: hipMemcpyAsync on the stream (mode 0).
// 16 x ResNet-34 bf16 back to back 134.5 -> 117.7 us, one call on an idle GPU 146.5 -> 139 us;
// 64 x ResNet-8 225 -> 205 us; 128 x ResNet-34 bf16 894 -> 851 us; the small rounds unchanged
// (profiles/r05d, r05f, r05g).
__global__ __launch_bounds__(256) void table_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                         int64_t n16) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n16;
       i += static_cast<int64_t>(gridDim.x) * 256)
    dst[i] = src[i];
}

constexpr int64_t kTableSideCopyMinBytes = int64_t{256} << 20;
std::map<int, hipStream_t> g_table_streams;  // device -> side stream of the table uploads (dla_shutdown frees)

// Is the reduce's stream still busy with the table reduces this library queued on it — will it be when a
// side copy started now has finished?  Estimated on the host from the work queued (its algorithmic bytes at
// 6 TB/s, the table kernel's measured rate), not asked of the runtime: hipStreamQuery costs ~4 us of GPU
// time between the kernels (profiles/r05g: 120.2 vs 115.8 us start to start, 16 x ResNet-34).  Work other
// than this library's on the stream is not seen: such a stream counts as idle (the copy kernel, correct
// and 4-6 us slower back to back).
struct StreamClock {
  std::chrono::steady_clock::time_point busy_until;
};
std::mutex g_clock_mu;
std::map<hipStream_t, StreamClock> g_stream_clock;

bool stream_busy_through(hipStream_t s, int64_t moved) {
  using clk = std::chrono::steady_clock;
  constexpr double kBytesPerUs = 6.0e6;                   // ~6 TB/s
  const auto side_copy = std::chrono::microseconds(25);  // side copy + the host's wait for it
  const auto now = clk::now();
  std::lock_guard<std::mutex> lock(g_clock_mu);
  if (g_stream_clock.size() > 64) g_stream_clock.clear();  // streams come and go: keep the map small
  StreamClock& c = g_stream_clock[s];
  const bool busy = c.busy_until > now + side_copy;
  const auto start = busy ? c.busy_until : now + side_copy;
  c.busy_until = start + std::chrono::microseconds(static_cast<int64_t>(static_cast<double>(moved) / kBytesPerUs));
  return busy;
}

int table_copy_mode() {  // -1 = the policy; the tuning build's DLA_TABLE_COPY forces 0..3
  static const int mode = [] {
    const char* v = tuning_env("DLA_TABLE_COPY");
    return v ? std::atoi(v) : -1;
  }();
  return mode;
}

hipError_t upload_table(char* td, const char* th, size_t bytes, int64_t moved, hipStream_t s) {
  const bool mapped = (bytes & 15u) == 0 && is_mapped_host_ptr(th);
  int mode = table_copy_mode();
  if (mode < 0) mode = (moved >= kTableSideCopyMinBytes && stream_busy_through(s, moved)) ? 3 : mapped ? 1 : 0;
  if (mode == 1 && mapped) {
    const int64_t n16 = static_cast<int64_t>(bytes / 16);
    int64_t grid = (n16 + 255) / 256;
    if (grid > 256) grid = 256;
    hipLaunchKernelGGL(table_copy_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), 0, s,
                       reinterpret_cast<const uint4*>(th), reinterpret_cast<uint4*>(td), n16);
    return hipGetLastError();
  }
  if (mode == 2 || mode == 3) {
    int dev = -1;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::unique_lock<std::mutex> lock(g_shard_mu);
    hipStream_t& side = g_table_streams[dev];
    if (!side && (e = hipStreamCreateWithFlags(&side, hipStreamNonBlocking)) != hipSuccess) return e;
    hipEvent_t ev;
    if ((e = take_event(dev, &ev)) != hipSuccess) return e;
    const hipStream_t side_s = side;
    lock.unlock();
    e = hipMemcpyAsync(td, th, bytes, hipMemcpyHostToDevice, side_s);
    if (e == hipSuccess) e = hipEventRecord(ev, side_s);
    if (e == hipSuccess) e = mode == 2 ? hipStreamWaitEvent(s, ev, 0) : hipEventSynchronize(ev);
    lock.lock();
    g_event_pool.push_back({dev, ev});  // reusable once recorded: a stream wait holds its own reference
    return e;
  }
  return hipMemcpyAsync(td, th, bytes, hipMemcpyHostToDevice, s);
}

int wsum_sharded_impl(int dtype, int n_shards, const int* dev_ids, const void* const* peers, const double* weights,
                      int n_peers, int64_t n_elems, void* const* outs, int gather, void* const* streams) {
  g_last_error.clear();
  const int es = elem_size(dtype);
  if (es == 0) return fail(DLA_E_INVALID, "dla_wsum_sharded: unknown dtype " + std::to_string(dtype));
  if (n_shards < 1 || !dev_ids || !outs || !streams)
    return fail(DLA_E_INVALID, "dla_wsum_sharded: need n_shards >= 1 and dev_ids / outs / streams arrays");
  if (n_peers < 1 || !peers || !weights)
    return fail(DLA_E_INVALID, "dla_wsum_sharded: n_peers must be >= 1 (fedavg.py:20 indexes models[0])");
  if (n_elems < 0) return fail(DLA_E_INVALID, "dla_wsum_sharded: n_elems < 0");
  if (gather < 0 || gather > 2) return fail(DLA_E_INVALID, "dla_wsum_sharded: gather must be 0, 1 or 2");
  if (n_elems == 0) return DLA_OK;
  int n_dev = 0;
  if (hipGetDeviceCount(&n_dev) != hipSuccess) return fail(DLA_E_INVALID, "dla_wsum_sharded: no HIP device");
  for (int s = 0; s < n_shards; ++s) {
    if (dev_ids[s] < 0 || dev_ids[s] >= n_dev)
      return fail(DLA_E_INVALID, "dla_wsum_sharded: bad device id for shard " + std::to_string(s));
    if (!outs[s]) return fail(DLA_E_INVALID, "dla_wsum_sharded: null out for shard " + std::to_string(s));
  }
  for (int k = 0; k < n_peers; ++k)
    if (!peers[k]) return fail(DLA_E_INVALID, "dla_wsum_sharded: null peer pointer " + std::to_string(k));
  const int64_t per = shard_bucket_elems(es, n_elems, n_shards);
  std::lock_guard<std::mutex> lock(g_shard_mu);
  DeviceGuard guard;
  // peer access: every shard's GPU reads every peer and writes its own output(s)
  std::vector<int> owners(static_cast<size_t>(n_peers));
  for (int k = 0; k < n_peers; ++k) owners[k] = owner_device(peers[k]);
  std::vector<int> out_owner(static_cast<size_t>(n_shards));
  for (int s = 0; s < n_shards; ++s) out_owner[s] = owner_device(outs[s]);
  for (int s = 0; s < n_shards; ++s) {
    const int dev = dev_ids[s];
    hipError_t e = hipSetDevice(dev);
    for (int k = 0; e == hipSuccess && k < n_peers; ++k) e = ensure_peer_access(dev, owners[k]);
    if (e == hipSuccess) e = ensure_peer_access(dev, out_owner[s]);
    if (e != hipSuccess)
      return fail(static_cast<int>(e), std::string("dla_wsum_sharded: peer access for shard ") + std::to_string(s) +
                                           ": " + hipGetErrorString(e));
  }
  // the reduce of every bucket, each on its own GPU and stream
  const Launch l = resolve(nullptr);
  std::vector<const void*> shifted(static_cast<size_t>(n_peers));
  for (int s = 0; s < n_shards; ++s) {
    const int64_t b = per * s < n_elems ? per * s : n_elems;
    const int64_t e_ = per * (s + 1) < n_elems ? per * (s + 1) : n_elems;
    if (b >= e_) continue;
    for (int k = 0; k < n_peers; ++k) shifted[k] = static_cast<const char*>(peers[k]) + b * es;
    void* o = static_cast<char*>(outs[s]) + b * es;
    if (n_peers > kMaxPeersPerPass)  // multi-pass: out carries the running sum (as dla_wsum)
      for (int k = 1; k < n_peers; ++k)
        if (shifted[k] == o)
          return fail(DLA_E_ALIAS, "dla_wsum_sharded: out of shard " + std::to_string(s) + " aliases peer " +
                                       std::to_string(k));
    hipError_t e = hipSetDevice(dev_ids[s]);
    if (e == hipSuccess) {
      hipStream_t st = static_cast<hipStream_t>(streams[s]);
      switch (dtype) {
        case DLA_F32: e = run<DLA_F32>(shifted.data(), weights, n_peers, e_ - b, o, st, l); break;
        case DLA_BF16: e = run<DLA_BF16>(shifted.data(), weights, n_peers, e_ - b, o, st, l); break;
        case DLA_F16: e = run<DLA_F16>(shifted.data(), weights, n_peers, e_ - b, o, st, l); break;
        default: e = run<DLA_F64>(shifted.data(), weights, n_peers, e_ - b, o, st, l); break;
      }
    }
    if (e != hipSuccess)
      return fail(static_cast<int>(e), std::string("dla_wsum_sharded: shard ") + std::to_string(s) + ": " +
                                           hipGetErrorString(e));
  }
  if (gather == 0) return DLA_OK;
  // gather: bucket s (on outs[s]) -> outs[d] for every other destination d (1) or d = 0 only (2),
  // enqueued on the destination's stream after an event recorded behind shard s's reduce
  std::vector<hipEvent_t> done(static_cast<size_t>(n_shards), nullptr);
  hipError_t e = hipSuccess;
  for (int s = 0; e == hipSuccess && s < n_shards; ++s) {
    e = hipSetDevice(dev_ids[s]);
    if (e == hipSuccess) e = take_event(dev_ids[s], &done[s]);
    if (e == hipSuccess) e = hipEventRecord(done[s], static_cast<hipStream_t>(streams[s]));
  }
  const int n_dst = gather == 1 ? n_shards : 1;
  for (int d = 0; e == hipSuccess && d < n_dst; ++d) {
    e = hipSetDevice(dev_ids[d]);
    hipStream_t sd = static_cast<hipStream_t>(streams[d]);
    for (int s = 0; e == hipSuccess && s < n_shards; ++s) {
      const int64_t b = per * s < n_elems ? per * s : n_elems;
      const int64_t e_ = per * (s + 1) < n_elems ? per * (s + 1) : n_elems;
      if (s == d || b >= e_ || outs[s] == outs[d]) continue;  // same buffer: the bucket is already there
      e = hipStreamWaitEvent(sd, done[s], 0);
      if (e == hipSuccess)
        e = hipMemcpyPeerAsync(static_cast<char*>(outs[d]) + b * es, dev_ids[d],
                               static_cast<const char*>(outs[s]) + b * es, dev_ids[s],
                               static_cast<size_t>((e_ - b) * es), sd);
    }
  }
  for (int s = 0; s < n_shards; ++s)  // an event may be re-recorded once every wait on it is enqueued
    if (done[s]) g_event_pool.push_back({dev_ids[s], done[s]});
  if (e != hipSuccess) return fail(static_cast<int>(e), std::string("dla_wsum_sharded: gather: ") + hipGetErrorString(e));
  return DLA_OK;
}

// Threads for one dla_host_copy_batch: one per 2 MiB up to DLA_COPY_THREADS (default 8; the GPU
// box's CPU share is 16); batches under 4 MiB stay on the calling thread.
int copy_threads(int64_t total) {
  static const int cap = [] {
    const char* e = tuning_env("DLA_COPY_THREADS");
    const int v = e ? std::atoi(e) : 8;
    return v < 1 ? 1 : v > 64 ? 64 : v;
  }();
  const int64_t by_size = total >> 21;
  return static_cast<int>(by_size < 2 ? 1 : by_size < cap ? by_size : cap);
}

// Persistent copy workers.  dla_host_reduce packs every chunk of a round (hundreds of chunks for
// the 128-peer google_speech round), so threads spawned per call (10-20 us each) would add up.
// One round at a time runs on the pool; a concurrent caller (the bucket-sharded host path runs one
// host thread per GPU) spawns its own threads instead.  The pool is never destroyed: its workers
// sleep on the condition variable until the process exits.
class CopyPool {
 public:
  // fn(0) on the calling thread and fn(1..n-1) on workers; false if another round holds the pool.
  template <typename F>
  bool try_run(int n, F& fn) {
    // a forked child has the pool's bookkeeping but none of its threads: it spawns its own
    if (getpid() != pid_) return false;
    std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
    if (!busy.owns_lock()) return false;
    std::function<void(int)> task = [&fn](int t) { fn(t); };
    {
      std::lock_guard<std::mutex> g(mu_);
      while (static_cast<int>(workers_.size()) < n - 1) workers_.emplace_back([this] { loop(); });
      task_ = &task;
      n_ = n;
      next_ = 1;
      pending_ = n - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [this] { return pending_ == 0; });
    task_ = nullptr;
    return true;
  }

 private:
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> g(mu_);
    for (;;) {
      cv_.wait(g, [&] { return gen_ != seen; });
      seen = gen_;
      while (task_ && next_ < n_) {
        const int t = next_++;
        const std::function<void(int)>* f = task_;
        g.unlock();
        (*f)(t);
        g.lock();
        if (--pending_ == 0) done_cv_.notify_one();
      }
    }
  }
  const pid_t pid_ = getpid();
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  const std::function<void(int)>* task_ = nullptr;
  int n_ = 0, next_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
};

CopyPool& copy_pool() {
  static CopyPool* pool = new CopyPool;  // leaked on purpose: no join at exit
  return *pool;
}

// Streaming (non-temporal) host copy for packs into page-locked staging that only the GPU reads next
// (a DMA or the kernel across PCIe): 32-byte vmovnt stores go straight to DRAM, with no read for
// ownership of the destination lines and no eviction of the packing thread's cache.
typedef long long v4i64 __attribute__((vector_size(32)));
__attribute__((target("avx2"))) void stream_copy_avx2(char* d, const char* s, size_t n) {
  size_t head = (32 - (reinterpret_cast<uintptr_t>(d) & 31)) & 31;
  if (head > n) head = n;
  std::memcpy(d, s, head);
  d += head, s += head, n -= head;
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    v4i64 a, b, c, e;
    std::memcpy(&a, s + i, 32), std::memcpy(&b, s + i + 32, 32);
    std::memcpy(&c, s + i + 64, 32), std::memcpy(&e, s + i + 96, 32);
    __builtin_nontemporal_store(a, reinterpret_cast<v4i64*>(d + i));
    __builtin_nontemporal_store(b, reinterpret_cast<v4i64*>(d + i + 32));
    __builtin_nontemporal_store(c, reinterpret_cast<v4i64*>(d + i + 64));
    __builtin_nontemporal_store(e, reinterpret_cast<v4i64*>(d + i + 96));
  }
  std::memcpy(d + i, s + i, n - i);
}

// DLA_COPY_NT=0 turns the streaming stores off (A/B); they need AVX2 (every MI355X host has it).
bool stream_copies() {
  static const bool on = [] {
    const char* e = tuning_env("DLA_COPY_NT");
    return !(e && std::atoi(e) == 0) && __builtin_cpu_supports("avx2");
  }();
  return on;
}

inline void copy_bytes(void* d, const void* s, int64_t n, bool nt) {
  if (nt && n >= 4096)
    stream_copy_avx2(static_cast<char*>(d), static_cast<const char*>(s), static_cast<size_t>(n));
  else
    std::memcpy(d, s, static_cast<size_t>(n));
}

// dsts[i] <- srcs[i], bytes[i] each (validated by the caller); threaded from 4 MiB.  nt: streaming
// stores (packs into page-locked staging read by the GPU next), fenced before the call returns.
// min_threads: at least this many threads from 256 KiB per thread on (a copy on the critical path:
// the last chunk's unpack, which nothing else overlaps).
void copy_batch(void* const* dsts, const void* const* srcs, const int64_t* bytes, int n, bool nt = false,
                int min_threads = 1) {
  nt = nt && stream_copies();
  int64_t total = 0;
  for (int i = 0; i < n; ++i) total += bytes[i];
  int threads = copy_threads(total);
  if (min_threads > threads) {
    const int64_t by_quarter_mib = total >> 18;
    threads = static_cast<int>(by_quarter_mib < min_threads ? (by_quarter_mib < threads ? threads : by_quarter_mib)
                                                            : min_threads);
  }
  if (threads <= 1) {
    for (int i = 0; i < n; ++i)
      if (bytes[i] > 0) copy_bytes(dsts[i], srcs[i], bytes[i], nt);
    if (nt) __builtin_ia32_sfence();
    return;
  }
  // Large batches (an EVA block list gathered into a page-locked ingress buffer: ~1 700
  // blocks per 100 MB model) split into equal byte ranges, one per thread; a range may start
  // or end inside a segment.
  auto copy_range = [&](int64_t lo, int64_t hi) {
    int64_t off = 0;
    for (int i = 0; i < n && off < hi; off += bytes[i], ++i) {
      const int64_t s0 = lo > off ? lo : off, e0 = hi < off + bytes[i] ? hi : off + bytes[i];
      if (s0 < e0)
        copy_bytes(static_cast<char*>(dsts[i]) + (s0 - off), static_cast<const char*>(srcs[i]) + (s0 - off), e0 - s0,
                   nt);
    }
    if (nt) __builtin_ia32_sfence();  // this thread's streaming stores are visible before it reports done
  };
  const int64_t per = (total + threads - 1) / threads;
  auto part = [&](int t) { copy_range(per * t < total ? per * t : total, per * (t + 1) < total ? per * (t + 1) : total); };
  if (copy_pool().try_run(threads, part)) return;
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(part, t);
  part(0);
  for (auto& th : pool) th.join();
}

}  // namespace

struct dla_plan {
  int dtype;
  std::vector<const void*> peers;
  std::vector<double> weights;
  int64_t n_elems;
  void* out;
  dla_launch_cfg_t cfg;
  bool has_cfg;
};

extern "C" {

int dla_version(void) { return DLA_ABI_VERSION; }

const char* dla_build_id(void) { return kBuildIdTag + sizeof("dlagg-build-id:") - 1; }

const char* dla_last_error(void) { return g_last_error.c_str(); }

int dla_max_peers_per_pass(void) { return kMaxPeersPerPass; }

const char* dla_select_kernel(int dtype, int n_peers, int64_t n_elems) {
  const int es = elem_size(dtype);
  if (es == 0 || n_peers < 1 || n_elems < 0) return "";
  const int e = 16 / es;  // elements per 16-byte chunk
  const int first_pass = n_peers < kMaxPeersPerPass ? n_peers : kMaxPeersPerPass;
  if ((dtype == DLA_BF16 || dtype == DLA_F16) && first_pass <= 8) return "wsum_vec_kernel";
  if (dtype != DLA_F64 && first_pass > 8 &&
      !(dtype == DLA_F32 && (first_pass == 16 || first_pass == 32) && use_bigtile(n_elems / e, e, n_peers)))
    return "wsum_vec_kernel";
  if (use_wide(n_elems / e, first_pass, e)) return "wsum_wide_kernel";
  if (dtype == DLA_F32 && n_peers == 8 && int64_t{8} * n_elems * 4 >= kMallBytes) return "wsum_vec_kernel";
  if ((dtype == DLA_F32 || dtype == DLA_F64) && use_bigtile(n_elems / e, e, n_peers))
    return "wsum_bigtile_kernel";
  return "wsum_stream_kernel";
}

int dla_wsum(int dtype, const void* const* peers, const double* weights, int n_peers, int64_t n_elems,
             void* out, void* stream) {
  return wsum_impl(dtype, peers, weights, n_peers, n_elems, out, stream, nullptr);
}

int dla_wsum_ex(int dtype, const void* const* peers, const double* weights, int n_peers,
                int64_t n_elems, void* out, void* stream, const dla_launch_cfg_t* cfg) {
  return wsum_impl(dtype, peers, weights, n_peers, n_elems, out, stream, cfg);
}

int dla_wsum_slab(int dtype, const void* base, int64_t pitch_elems, const double* weights, int n_peers,
                  int64_t n_elems, void* out, void* stream) {
  g_last_error.clear();
  const int es = elem_size(dtype);
  if (es == 0) return fail(DLA_E_INVALID, "dla_wsum_slab: unknown dtype");
  if (!base || n_peers < 1 || pitch_elems < n_elems)
    return fail(DLA_E_INVALID, "dla_wsum_slab: need base, n_peers >= 1 and pitch_elems >= n_elems");
  std::string ptrs;  // small host table of row pointers
  ptrs.resize(sizeof(void*) * static_cast<size_t>(n_peers));
  const void** rows = reinterpret_cast<const void**>(&ptrs[0]);
  for (int k = 0; k < n_peers; ++k)
    rows[k] = static_cast<const char*>(base) + static_cast<int64_t>(k) * pitch_elems * es;
  return wsum_impl(dtype, rows, weights, n_peers, n_elems, out, stream, nullptr);
}

int dla_wsum_multi(int dtype, int n_tensors, const void* const* peer_ptrs, void* const* outs,
                   const int64_t* numels, const double* weights, int n_peers, void* stream) {
  g_last_error.clear();
  if (n_tensors < 0 || (n_tensors > 0 && (!peer_ptrs || !outs || !numels)))
    return fail(DLA_E_INVALID, "dla_wsum_multi: bad tensor table");
  const int es = elem_size(dtype);
  if (es == 0) return fail(DLA_E_INVALID, "dla_wsum_multi: unknown dtype " + std::to_string(dtype));
  if (n_peers < 1 || !weights) return fail(DLA_E_INVALID, "dla_wsum_multi: n_peers must be >= 1");
  // Small, 16-byte aligned tensors share launches (<= 32 peers); large or unaligned
  // tensors, and passes of more peers, take the single-tensor path.
  constexpr int64_t kOwnLaunchBytes = 32ll << 20;
  std::vector<int> packed;
  for (int t = 0; t < n_tensors; ++t) {
    if (numels[t] < 0) return fail(DLA_E_INVALID, "dla_wsum_multi: negative numel");
    if (numels[t] == 0) continue;
    bool ok = n_peers <= 32 && numels[t] * es < kOwnLaunchBytes && outs[t] &&
              (reinterpret_cast<uintptr_t>(outs[t]) & 15u) == 0;
    for (int k = 0; ok && k < n_peers; ++k) {
      const void* q = peer_ptrs[static_cast<int64_t>(t) * n_peers + k];
      ok = q && (reinterpret_cast<uintptr_t>(q) & 15u) == 0;
    }
    if (ok) {
      packed.push_back(t);
      continue;
    }
    const int rc = wsum_impl(dtype, peer_ptrs + static_cast<int64_t>(t) * n_peers, weights, n_peers, numels[t],
                             outs[t], stream, nullptr);
    if (rc != DLA_OK) return rc;
  }
  if (packed.empty()) return DLA_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e;
  switch (dtype) {
    case DLA_F32: e = run_multi_dt<DLA_F32>(packed, peer_ptrs, outs, numels, weights, n_peers, s); break;
    case DLA_BF16: e = run_multi_dt<DLA_BF16>(packed, peer_ptrs, outs, numels, weights, n_peers, s); break;
    case DLA_F16: e = run_multi_dt<DLA_F16>(packed, peer_ptrs, outs, numels, weights, n_peers, s); break;
    default: e = run_multi_dt<DLA_F64>(packed, peer_ptrs, outs, numels, weights, n_peers, s); break;
  }
  if (e != hipSuccess) return fail(static_cast<int>(e), std::string("dla_wsum_multi: ") + hipGetErrorString(e));
  return DLA_OK;
}

int64_t dla_wsum_multi_table_bytes(int n_tensors, int n_peers) {
  if (n_tensors < 0 || n_peers < 1) return 0;
  return multi_table_bytes(n_tensors, n_peers);
}

namespace {
int multi_table_impl(int dtype, int n_tensors, const void* const* peer_ptrs, void* const* outs,
                     const int64_t* numels, const double* weights, int n_peers, bool acc_in, void* table_host,
                     void* table_dev, void* stream) {
  g_last_error.clear();
  if (n_tensors < 0 || (n_tensors > 0 && (!peer_ptrs || !outs || !numels)))
    return fail(DLA_E_INVALID, "dla_wsum_multi_table: bad tensor table");
  const int es = elem_size(dtype);
  if (es == 0) return fail(DLA_E_INVALID, "dla_wsum_multi_table: unknown dtype " + std::to_string(dtype));
  if (n_peers < 1 || !weights) return fail(DLA_E_INVALID, "dla_wsum_multi_table: n_peers must be >= 1");
  std::vector<int> packed;
  for (int t = 0; t < n_tensors; ++t) {
    if (numels[t] < 0) return fail(DLA_E_INVALID, "dla_wsum_multi_table: negative numel");
    if (numels[t] == 0) continue;
    const void* const* row = peer_ptrs + static_cast<int64_t>(t) * n_peers;
    bool ok = dtype != DLA_F64 && outs[t] && (reinterpret_cast<uintptr_t>(outs[t]) & 15u) == 0;
    for (int k = 0; ok && k < n_peers; ++k) ok = row[k] && (reinterpret_cast<uintptr_t>(row[k]) & 15u) == 0;
    if (ok && acc_in)  // out carries the running sum from the start (as dla_wsum with acc_in)
      for (int k = 0; k < n_peers; ++k)
        if (row[k] == outs[t])
          return fail(DLA_E_ALIAS, "dla_wsum_multi_table_acc: out of tensor " + std::to_string(t) + " aliases peer " +
                                       std::to_string(k));
    if (ok && !acc_in && n_peers > kMaxPeersPerPass)  // multi-pass: out carries the running sum (as dla_wsum)
      for (int k = 1; ok && k < n_peers; ++k)
        if (row[k] == outs[t])
          return fail(DLA_E_ALIAS, "dla_wsum_multi_table: out of tensor " + std::to_string(t) + " aliases peer " +
                                       std::to_string(k) + "; only peers[0] may alias out when n_peers > " +
                                       std::to_string(kMaxPeersPerPass));
    if (ok) {
      packed.push_back(t);
      continue;
    }
    const int rc = wsum_impl(dtype, row, weights, n_peers, numels[t], outs[t], stream, nullptr, acc_in);
    if (rc != DLA_OK) return rc;
  }
  if (packed.empty()) return DLA_OK;
  if (!table_host || !table_dev) return fail(DLA_E_INVALID, "dla_wsum_multi_table: null table buffer");
  if (!is_pinned_host_ptr(table_host))
    return fail(DLA_E_INVALID, "dla_wsum_multi_table: table_host must be page-locked host memory (hipHostMalloc)");
  if (!is_device_ptr(table_dev)) return fail(DLA_E_INVALID, "dla_wsum_multi_table: table_dev must be device memory");
  if ((reinterpret_cast<uintptr_t>(table_host) & 15u) || (reinterpret_cast<uintptr_t>(table_dev) & 15u))
    return fail(DLA_E_INVALID, "dla_wsum_multi_table: table buffers must be 16-byte aligned");
  // The table's upload keys its side stream, its event and the mapped-table check on the current device:
  // make that the device holding table_dev (the reduce's device) for this call, whatever the caller had
  // current (models reduced on cuda:1 while device 0 is current).
  DeviceGuard guard;
  const int tdev = owner_device(table_dev);
  int cur = -1;
  if (tdev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != tdev && hipSetDevice(tdev) != hipSuccess)
    return fail(DLA_E_INVALID, "dla_wsum_multi_table: cannot select the table's device " + std::to_string(tdev));
  hipStream_t s = static_cast<hipStream_t>(stream);
  char* th = static_cast<char*>(table_host);
  char* td = static_cast<char*>(table_dev);
  hipError_t e;
  switch (dtype) {
    case DLA_F32: e = run_multi_table<DLA_F32>(packed, peer_ptrs, outs, numels, weights, n_peers, th, td, s, acc_in); break;
    case DLA_BF16: e = run_multi_table<DLA_BF16>(packed, peer_ptrs, outs, numels, weights, n_peers, th, td, s, acc_in); break;
    default: e = run_multi_table<DLA_F16>(packed, peer_ptrs, outs, numels, weights, n_peers, th, td, s, acc_in); break;
  }
  if (e != hipSuccess) return fail(static_cast<int>(e), std::string("dla_wsum_multi_table: ") + hipGetErrorString(e));
  return DLA_OK;
}
}  // namespace

int dla_wsum_multi_table(int dtype, int n_tensors, const void* const* peer_ptrs, void* const* outs,
                         const int64_t* numels, const double* weights, int n_peers, void* table_host,
                         void* table_dev, void* stream) {
  return multi_table_impl(dtype, n_tensors, peer_ptrs, outs, numels, weights, n_peers, false, table_host, table_dev,
                          stream);
}

int dla_wsum_multi_table_acc(int dtype, int n_tensors, const void* const* peer_ptrs, void* const* outs,
                             const int64_t* numels, const double* weights, int n_peers, int acc_in, void* table_host,
                             void* table_dev, void* stream) {
  return multi_table_impl(dtype, n_tensors, peer_ptrs, outs, numels, weights, n_peers, acc_in != 0, table_host,
                          table_dev, stream);
}

int dla_plan_create(dla_plan_t** plan, int dtype, const void* const* peers, const double* weights, int n_peers,
                    int64_t n_elems, void* out, const dla_launch_cfg_t* cfg) {
  g_last_error.clear();
  if (!plan) return fail(DLA_E_INVALID, "dla_plan_create: null plan");
  *plan = nullptr;
  if (elem_size(dtype) == 0) return fail(DLA_E_INVALID, "dla_plan_create: unknown dtype");
  if (n_peers < 1 || !peers || !weights || n_elems < 0 || (n_elems > 0 && !out))
    return fail(DLA_E_INVALID, "dla_plan_create: bad arguments");
  for (int k = 0; k < n_peers; ++k)
    if (!peers[k]) return fail(DLA_E_INVALID, "dla_plan_create: null peer pointer");
  dla_plan* p = new (std::nothrow) dla_plan;
  if (!p) return fail(DLA_E_INVALID, "dla_plan_create: out of host memory");
  p->dtype = dtype;
  p->peers.assign(peers, peers + n_peers);
  p->weights.assign(weights, weights + n_peers);
  p->n_elems = n_elems;
  p->out = out;
  p->has_cfg = cfg != nullptr;
  if (cfg) p->cfg = *cfg;
  *plan = p;
  return DLA_OK;
}

int dla_plan_set_weights(dla_plan_t* plan, const double* weights) {
  g_last_error.clear();
  if (!plan || !weights) return fail(DLA_E_INVALID, "dla_plan_set_weights: null argument");
  std::memcpy(plan->weights.data(), weights, sizeof(double) * plan->weights.size());
  return DLA_OK;
}

int dla_plan_launch(const dla_plan_t* plan, void* stream) {
  if (!plan) return fail(DLA_E_INVALID, "dla_plan_launch: null plan");
  return wsum_impl(plan->dtype, plan->peers.data(), plan->weights.data(), static_cast<int>(plan->peers.size()),
                   plan->n_elems, plan->out, stream, plan->has_cfg ? &plan->cfg : nullptr);
}

void dla_plan_destroy(dla_plan_t* plan) { delete plan; }

int dla_mean(int dtype, const void* const* peers, int n_peers, int64_t n_elems, void* out, void* stream) {
  g_last_error.clear();
  if (dtype != DLA_F32 && dtype != DLA_F64) return fail(DLA_E_INVALID, "dla_mean: F32 or F64 only");
  if (n_peers < 1 || !peers) return fail(DLA_E_INVALID, "dla_mean: n_peers must be >= 1");
  if (n_elems < 0) return fail(DLA_E_INVALID, "dla_mean: n_elems < 0");
  if (n_elems == 0) return DLA_OK;
  if (!out) return fail(DLA_E_INVALID, "dla_mean: null out");
  for (int k = 0; k < n_peers; ++k) {
    if (!peers[k]) return fail(DLA_E_INVALID, "dla_mean: null peer pointer");
    if (n_peers > kMaxPeersPerPass && k > 0 && peers[k] == out)
      return fail(DLA_E_ALIAS, "dla_mean: out aliases a peer other than peers[0] in a multi-pass mean");
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  const hipError_t e = dtype == DLA_F32 ? run_mean<DLA_F32>(peers, n_peers, n_elems, out, s)
                                        : run_mean<DLA_F64>(peers, n_peers, n_elems, out, s);
  if (e != hipSuccess) return fail(static_cast<int>(e), std::string("dla_mean: ") + hipGetErrorString(e));
  return DLA_OK;
}

int dla_wsum_mixed(int out_dtype, const int* peer_dtypes, const void* const* peers, const double* weights,
                   int n_peers, int64_t n_elems, void* out, void* stream) {
  g_last_error.clear();
  if (elem_size(out_dtype) == 0) return fail(DLA_E_INVALID, "dla_wsum_mixed: unknown out dtype");
  if (n_peers < 1 || !peers || !weights || !peer_dtypes)
    return fail(DLA_E_INVALID, "dla_wsum_mixed: n_peers must be >= 1 with peers, weights and dtypes");
  if (n_elems < 0) return fail(DLA_E_INVALID, "dla_wsum_mixed: n_elems < 0");
  for (int k = 0; k < n_peers; ++k)
    if (elem_size(peer_dtypes[k]) == 0)
      return fail(DLA_E_INVALID, "dla_wsum_mixed: unknown dtype of peer " + std::to_string(k));
  if (peer_dtypes[0] != out_dtype)
    return fail(DLA_E_INVALID, "dla_wsum_mixed: peers[0] is models[0], whose deepcopy is the result: "
                               "its dtype must be out_dtype (fedavg.py:20)");
  if (n_elems == 0) return DLA_OK;  // a 0-element parameter: its tensors may carry null pointers
  for (int k = 0; k < n_peers; ++k)
    if (!peers[k]) return fail(DLA_E_INVALID, "dla_wsum_mixed: null peer pointer " + std::to_string(k));
  if (!out) return fail(DLA_E_INVALID, "dla_wsum_mixed: null out");
  for (int k = 1; k < n_peers; ++k)
    if (peers[k] == out) return fail(DLA_E_ALIAS, "dla_wsum_mixed: out aliases peer " + std::to_string(k));
  const hipError_t e = run_mixed(out_dtype, peer_dtypes, peers, weights, n_peers, n_elems, out,
                                 static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return fail(static_cast<int>(e), std::string("dla_wsum_mixed: ") + hipGetErrorString(e));
  return DLA_OK;
}

int dla_host_copy_batch(void* const* dsts, const void* const* srcs, const int64_t* bytes, int n) {
  return dla_host_copy_batch_ex(dsts, srcs, bytes, n, 0);
}

int dla_host_copy_batch_ex(void* const* dsts, const void* const* srcs, const int64_t* bytes, int n, int flags) {
  g_last_error.clear();
  if (flags & ~DLA_COPY_STREAMING) return fail(DLA_E_INVALID, "dla_host_copy_batch: unknown flags");
  if (n < 0 || (n > 0 && (!dsts || !srcs || !bytes))) return fail(DLA_E_INVALID, "dla_host_copy_batch: bad table");
  for (int i = 0; i < n; ++i) {
    if (bytes[i] < 0) return fail(DLA_E_INVALID, "dla_host_copy_batch: negative size at " + std::to_string(i));
    if (bytes[i] > 0 && (!dsts[i] || !srcs[i]))
      return fail(DLA_E_INVALID, "dla_host_copy_batch: null pointer at " + std::to_string(i));
  }
  copy_batch(dsts, srcs, bytes, n, (flags & DLA_COPY_STREAMING) != 0);
  return DLA_OK;
}

// The launch of a reduce that reads host memory across PCIe: the vector-per-lane kernel (n x 512 B of
// loads in flight per wave) — the shape-based choice (the 16-byte stream kernel for few fp32 peers) is
// tuned for HBM (r04e/r04f, dla_host_reduce).  fp64 keeps the shape-based choice (no vector kernel).
// Tuning build: DLA_HOST_AUTO_KERNEL=1 keeps the shape-based choice for host reads (A/B).
static const dla_launch_cfg_t* host_read_cfg(int dtype, int n_peers) {
  static const bool automatic = tuning_env("DLA_HOST_AUTO_KERNEL") != nullptr;
  if (automatic || dtype == DLA_F64) return nullptr;
  static thread_local dla_launch_cfg_t cfg;
  cfg = dla_launch_cfg_t{};
  cfg.variant = vec_variant(n_peers);
  return &cfg;
}

int dla_host_round_start(int dtype, int n_peers, int n_tensors, const void* const* tensors, const int64_t* numels,
                         const double* weights, void* rows, int64_t pitch_elems, void* result, void* stream) {
  g_last_error.clear();
  const int es = elem_size(dtype);
  if (es == 0) return fail(DLA_E_INVALID, "dla_host_round_start: unknown dtype");
  if (n_peers < 1 || n_tensors < 1 || !tensors || !numels || !weights || !rows || !result)
    return fail(DLA_E_INVALID, "dla_host_round_start: need n_peers >= 1, n_tensors >= 1 and every table");
  int64_t total = 0;
  for (int t = 0; t < n_tensors; ++t) {
    if (numels[t] < 0) return fail(DLA_E_INVALID, "dla_host_round_start: negative numel at " + std::to_string(t));
    total += numels[t];
  }
  if (pitch_elems < total || (pitch_elems * es) % 16)
    return fail(DLA_E_INVALID, "dla_host_round_start: pitch_elems must be >= sum(numels) and a multiple of 16 bytes");
  if ((reinterpret_cast<uintptr_t>(rows) & 15u) || (reinterpret_cast<uintptr_t>(result) & 15u))
    return fail(DLA_E_INVALID, "dla_host_round_start: rows and result must be 16-byte aligned");
  // The kernel reads `rows` and writes `result` across PCIe: both must be page-locked host memory
  // mapped into the device address space at the same address (hipHostMalloc / torch pin_memory).
  for (const void* p : {static_cast<const void*>(rows), static_cast<const void*>(result)}) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeHost || a.devicePointer != p) {
      (void)hipGetLastError();
      return fail(DLA_E_INVALID, "dla_host_round_start: rows / result must be page-locked host memory "
                                 "mapped for the device (hipHostMalloc)");
    }
  }
  for (int i = 0; i < n_peers * n_tensors; ++i)
    if (!tensors[i] && numels[i % n_tensors] > 0)
      return fail(DLA_E_INVALID, "dla_host_round_start: null tensor pointer at " + std::to_string(i));
  if (total == 0) return DLA_OK;
  {  // peers that already are page-locked rows: the kernel reads them where they are (no pack)
    std::vector<int64_t> start(n_tensors + 1, 0);
    for (int t = 0; t < n_tensors; ++t) start[t + 1] = start[t] + numels[t];
    std::vector<const char*> in_place;
    if (mapped_peer_rows(es, n_peers, n_tensors, tensors, start.data(), 0, total, in_place)) {
      g_host_in_place.fetch_add(1, std::memory_order_relaxed);
      std::vector<const void*> ptrs(in_place.begin(), in_place.end());
      return wsum_impl(dtype, ptrs.data(), weights, n_peers, total, result, stream, host_read_cfg(dtype, n_peers));
    }
  }
  // pack: tensor t of peer k -> row k at the tensor's flat offset (the zip order of fedavg.py:24)
  std::vector<void*> dsts(static_cast<size_t>(n_peers) * n_tensors);
  std::vector<const void*> srcs(dsts.size());
  std::vector<int64_t> bytes(dsts.size());
  std::vector<const void*> row_ptrs(n_peers);
  for (int k = 0; k < n_peers; ++k) {
    char* row = static_cast<char*>(rows) + static_cast<int64_t>(k) * pitch_elems * es;
    row_ptrs[k] = row;
    int64_t off = 0;
    for (int t = 0; t < n_tensors; ++t) {
      const size_t i = static_cast<size_t>(k) * n_tensors + t;
      dsts[i] = row + off;
      srcs[i] = tensors[i];
      bytes[i] = numels[t] * es;
      off += bytes[i];
    }
  }
  copy_batch(dsts.data(), srcs.data(), bytes.data(), static_cast<int>(dsts.size()), /*nt=*/true);
  const int rc = wsum_impl(dtype, row_ptrs.data(), weights, n_peers, total, result, stream, host_read_cfg(dtype, n_peers));
  return rc;
}

int dla_host_round_finish(int dtype, int n_tensors, const int64_t* numels, const void* result, void* const* outs,
                          void* stream) {
  g_last_error.clear();
  const int es = elem_size(dtype);
  if (es == 0) return fail(DLA_E_INVALID, "dla_host_round_finish: unknown dtype");
  if (n_tensors < 1 || !numels || !result || !outs)
    return fail(DLA_E_INVALID, "dla_host_round_finish: need n_tensors >= 1 and every table");
  for (int t = 0; t < n_tensors; ++t)
    if (numels[t] < 0 || (numels[t] > 0 && !outs[t]))
      return fail(DLA_E_INVALID, "dla_host_round_finish: bad tensor " + std::to_string(t));
  const hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return fail(static_cast<int>(e), std::string("dla_host_round_finish: ") + hipGetErrorString(e));
  // unpack: the averaged row -> the result's tensors (fedavg.py:25 lands in the deepcopy's params)
  std::vector<const void*> srcs(n_tensors);
  std::vector<int64_t> bytes(n_tensors);
  int64_t off = 0;
  for (int t = 0; t < n_tensors; ++t) {
    srcs[t] = static_cast<const char*>(result) + off;
    bytes[t] = numels[t] * es;
    off += bytes[t];
  }
  copy_batch(outs, srcs.data(), bytes.data(), n_tensors);
  return DLA_OK;
}

namespace {
struct Events {
  hipEvent_t e[6] = {};
  hipError_t create() {
    for (auto& x : e) {
      const hipError_t r = hipEventCreateWithFlags(&x, hipEventDisableTiming);
      if (r != hipSuccess) return r;
    }
    return hipSuccess;
  }
  ~Events() {
    for (auto x : e)
      if (x) (void)hipEventDestroy(x);
  }
};
}  // namespace

namespace {
// dla_host_reduce and dla_host_reduce_deferred: outs_ready == nullptr means outs[] is valid on entry;
// otherwise outs[] is read only once *outs_ready turns non-zero (> 0: filled; < 0: the caller gave up).
int host_reduce_impl(int dtype, int n_peers, int n_tensors, const void* const* tensors, const int64_t* numels,
                     const double* weights, void* const* outs, const int* outs_ready, int64_t begin, int64_t end,
                     int64_t chunk_elems, void* h_stage, void* d_stage, void* h_out, void* d_out, void* stream,
                     void* copy_stream) {
  g_last_error.clear();
  const int es = elem_size(dtype);
  if (es == 0) return fail(DLA_E_INVALID, "dla_host_reduce: unknown dtype");
  if (n_peers < 1 || n_tensors < 1 || !tensors || !numels || !weights || !outs || !h_stage || !d_stage || !h_out ||
      !d_out)
    return fail(DLA_E_INVALID, "dla_host_reduce: need n_peers >= 1, n_tensors >= 1 and every table and buffer");
  if (chunk_elems < 1 || (chunk_elems * es) % 256)
    return fail(DLA_E_INVALID, "dla_host_reduce: chunk_elems must be >= 1 and a multiple of 256 bytes");
  std::vector<int64_t> start(n_tensors + 1, 0);
  for (int t = 0; t < n_tensors; ++t) {
    if (numels[t] < 0) return fail(DLA_E_INVALID, "dla_host_reduce: negative numel at " + std::to_string(t));
    if (!outs_ready && numels[t] > 0 && !outs[t])
      return fail(DLA_E_INVALID, "dla_host_reduce: null output " + std::to_string(t));
    start[t + 1] = start[t] + numels[t];
  }
  for (int i = 0; i < n_peers * n_tensors; ++i)
    if (!tensors[i] && numels[i % n_tensors] > 0)
      return fail(DLA_E_INVALID, "dla_host_reduce: null tensor pointer at " + std::to_string(i));
  const int64_t total = start[n_tensors];
  if (begin < 0 || end < begin || end > total)
    return fail(DLA_E_INVALID, "dla_host_reduce: need 0 <= begin <= end <= sum(numels)");
  if (end == begin) return DLA_OK;
  if (!is_pinned_host_ptr(h_stage) || !is_pinned_host_ptr(h_out))
    return fail(DLA_E_INVALID, "dla_host_reduce: h_stage / h_out must be page-locked host memory (hipHostMalloc)");
  if (!is_device_ptr(d_stage) || !is_device_ptr(d_out))
    return fail(DLA_E_INVALID, "dla_host_reduce: d_stage / d_out must be device memory");
  const hipStream_t cs_ = static_cast<hipStream_t>(stream);
  const hipStream_t xs = static_cast<hipStream_t>(copy_stream);
  // Page-locked peer rows are read in place by the reduce (mapped_peer_rows: no pack, no H2D); its
  // output then goes straight into the page-locked h_out across PCIe when that is device-mapped too.
  std::vector<const char*> in_place;
  const bool mapped = mapped_peer_rows(es, n_peers, n_tensors, tensors, start.data(), begin, end, in_place);
  const bool out_mapped = mapped && is_mapped_host_ptr(h_out);
  if (mapped) g_host_in_place.fetch_add(1, std::memory_order_relaxed);
  // Pageable peers are packed into h_stage; when h_stage and h_out are device-mapped the reduce then
  // reads the packed rows across PCIe itself and writes h_out directly (no staging DMA either way; the
  // kernel's own PCIe reads ran at 57.3-57.6 GB/s against 51.7-57.0 for DMAs, profiles/r04a/
  // copy_probe.log).  Tuning build: DLA_HOST_STAGE_DMA=1 keeps the staging H2D / D2H DMAs (A/B).
  static const bool stage_dma = tuning_env("DLA_HOST_STAGE_DMA") != nullptr;
  const bool stage_read = !mapped && !stage_dma && is_mapped_host_ptr(h_stage) && is_mapped_host_ptr(h_out);
  // A reduce that reads host memory runs the vector-per-lane kernel (n x 512 B of loads in flight per
  // wave): the shape-based choice for 8 fp32 peers over a 32 MiB chunk is the 16-byte stream kernel,
  // whose fewer loads in flight suit HBM, not PCIe round trips (r04e: 8 x 25 M host round 17.9-20.4 ms
  // reading the packed rows with it, against 15.4-15.6 through the staging DMA).
  const dla_launch_cfg_t* read_cfg = host_read_cfg(dtype, n_peers);
  Events ev;  // h2d[2], red[2], d2h[2]
  hipError_t e = ev.create();
  if (e != hipSuccess) return fail(static_cast<int>(e), std::string("dla_host_reduce: ") + hipGetErrorString(e));
  hipEvent_t* h2d = ev.e;
  hipEvent_t* red = ev.e + 2;
  hipEvent_t* d2h = ev.e + 4;
  const int64_t row_bytes = chunk_elems * es;
  const int64_t buf_bytes = row_bytes * n_peers;
  // Chunk schedule: nothing crosses PCIe before the first chunk is packed, so the first chunks ramp
  // up (1/4, then 1/2 of chunk_elems, 256-byte multiples) and the pipeline fills in a quarter of the
  // time; then full chunks.  cs[c] .. cs[c + 1] are chunk c's flat elements.
  const int64_t align = 256 / es;
  std::vector<int64_t> cs{begin};
  // DLA_HOST_RAMP=k: the first chunk is 1/k of chunk_elems (a power of two; default 4; A/B knob)
  static const int64_t ramp = [] {
    const char* v = tuning_env("DLA_HOST_RAMP");
    int64_t r = v ? std::atoll(v) : 4;
    if (r < 1) r = 1;
    int64_t p = 1;
    while (p < r && p < 64) p *= 2;
    return p;
  }();
  for (int64_t part = ramp; cs.back() < end; part = part > 1 ? part / 2 : 1) {
    int64_t len = chunk_elems / part / align * align;
    if (len < align) len = align;
    cs.push_back(cs.back() + len < end ? cs.back() + len : end);
  }
  const int64_t n_chunks = static_cast<int64_t>(cs.size()) - 1;
  // Chunk c's rows are packed dense at pitch(c) (its length in bytes rounded up to 256, so every row
  // stays 16-byte aligned for the kernel): one contiguous H2D per chunk, the last one included.
  auto pitch = [&](int64_t c) { return ((cs[c + 1] - cs[c]) * es + 255) / 256 * 256; };
  std::vector<void*> dsts;
  std::vector<const void*> srcs;
  std::vector<int64_t> bytes;
  std::vector<const void*> rows(n_peers);
  // the tensors overlapping elements [c0, c1) of the flat (parameters()-order) vector
  auto pieces = [&](int64_t c0, int64_t c1, auto&& emit) {
    int t = static_cast<int>(std::upper_bound(start.begin(), start.end(), c0) - start.begin()) - 1;
    for (; t < n_tensors && start[t] < c1; ++t) {
      const int64_t a = c0 > start[t] ? c0 : start[t], b = c1 < start[t + 1] ? c1 : start[t + 1];
      if (a < b) emit(t, a, b);
    }
  };
  auto check = [&](hipError_t r, const char* what) {
    if (r != hipSuccess && e == hipSuccess) {
      e = r;
      g_last_error = std::string("dla_host_reduce: ") + what + ": " + hipGetErrorString(r);
    }
    return r == hipSuccess;
  };
  // Deferred outputs: the first unpack waits for the caller to publish outs[] (it allocates the
  // result's tensors while the first chunks are packed and copied in).  Acquire load: the caller's
  // stores into outs[] before its flag store are visible once the flag is.
  bool outs_known = outs_ready == nullptr;
  auto await_outs = [&]() {
    if (outs_known) return true;
    int v;
    while ((v = __atomic_load_n(outs_ready, __ATOMIC_ACQUIRE)) == 0) std::this_thread::yield();
    if (v < 0) {
      e = hipErrorInvalidValue;
      g_last_error = "dla_host_reduce: the caller abandoned the outputs";
      return false;
    }
    for (int t = 0; t < n_tensors; ++t)
      if (numels[t] > 0 && !outs[t]) {
        e = hipErrorInvalidValue;
        g_last_error = "dla_host_reduce: null output " + std::to_string(t);
        return false;
      }
    outs_known = true;
    return true;
  };
  // chunk c's averaged elements (h_out buffer c & 1) -> the result tensors (fedavg.py:25)
  auto unpack = [&](int64_t c, int min_threads) {
    const int buf = static_cast<int>(c & 1);
    if (!await_outs()) return;
    if (!check(hipEventSynchronize(d2h[buf]), "D2H")) return;
    const int64_t c0 = cs[c], c1 = cs[c + 1];
    dsts.clear(), srcs.clear(), bytes.clear();
    pieces(c0, c1, [&](int t, int64_t a, int64_t b) {
      dsts.push_back(static_cast<char*>(outs[t]) + (a - start[t]) * es);
      srcs.push_back(static_cast<const char*>(h_out) + buf * row_bytes + (a - c0) * es);
      bytes.push_back((b - a) * es);
    });
    copy_batch(dsts.data(), srcs.data(), bytes.data(), static_cast<int>(dsts.size()), false, min_threads);
  };
  // DLA_HOST_REDUCE_STATS=1: per-call phase times on stderr (host-path tuning)
  static const bool stats = tuning_env("DLA_HOST_REDUCE_STATS") != nullptr;
  using clk = std::chrono::steady_clock;
  double t_wait = 0, t_pack = 0, t_issue = 0, t_unpack = 0, t_first = 0;
  auto secs = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); };
  const auto t_start = clk::now();
  for (int64_t c = 0; c < n_chunks && e == hipSuccess; ++c) {
    const int buf = static_cast<int>(c & 1);
    const int64_t c0 = cs[c], c1 = cs[c + 1];
    const int64_t m = c1 - c0;
    const int64_t rp = pitch(c);
    const auto t0 = clk::now();
    char* hs = static_cast<char*>(h_stage) + buf * buf_bytes;
    char* ds = static_cast<char*>(d_stage) + buf * buf_bytes;
    char* dout = static_cast<char*>(d_out) + buf * row_bytes;
    char* hout = static_cast<char*>(h_out) + buf * row_bytes;
    if (mapped) {
      // the reduce reads chunk c of every peer's page-locked row across PCIe; h_out[buf] is free again
      // (chunk c-2's unpack ran on this thread during the previous iteration)
      for (int k = 0; k < n_peers; ++k) rows[k] = in_place[k] + c0 * es;
      const int rc = wsum_impl(dtype, rows.data(), weights, n_peers, m, out_mapped ? hout : dout, stream, read_cfg);
      if (rc != DLA_OK) {
        (void)hipStreamSynchronize(cs_);
        return rc;
      }
      if (!out_mapped && !check(hipMemcpyAsync(hout, dout, m * es, hipMemcpyDeviceToHost, cs_), "D2H")) break;
      if (!check(hipEventRecord(d2h[buf], cs_), "record")) break;
      const auto t3 = clk::now();
      if (c == 0) t_first = secs(t_start, t3);
      if (c >= 1) unpack(c - 1, 1);  // overlaps chunk c's reduce
      t_issue += secs(t0, t3), t_unpack += secs(t3, clk::now());
      continue;
    }
    // pack chunk c of every peer into row k of staging buffer `buf`, once the H2D of chunk c-2 has read it
    // (stage_read: once chunk c-2's reduce has; its unpack, which waited for it, ran last iteration)
    if (c >= 2 && !check(hipEventSynchronize(stage_read ? d2h[buf] : h2d[buf]), "H2D")) break;
    const auto t1 = clk::now();
    dsts.clear(), srcs.clear(), bytes.clear();
    for (int k = 0; k < n_peers; ++k) {
      rows[k] = (stage_read ? hs : ds) + k * rp;
      pieces(c0, c1, [&](int t, int64_t a, int64_t b) {
        dsts.push_back(hs + k * rp + (a - c0) * es);
        srcs.push_back(static_cast<const char*>(tensors[static_cast<size_t>(k) * n_tensors + t]) + (a - start[t]) * es);
        bytes.push_back((b - a) * es);
      });
    }
    copy_batch(dsts.data(), srcs.data(), bytes.data(), static_cast<int>(dsts.size()), /*nt=*/true);
    const auto t2 = clk::now();
    if (c == 0) t_first = secs(t_start, t2);
    if (stage_read) {  // the reduce reads the packed rows in h_stage[buf] and writes h_out[buf], across PCIe
      const int rc = wsum_impl(dtype, rows.data(), weights, n_peers, m, hout, stream, read_cfg);
      if (rc != DLA_OK) {
        (void)hipStreamSynchronize(cs_);
        return rc;
      }
      if (!check(hipEventRecord(d2h[buf], cs_), "record")) break;
      const auto t3 = clk::now();
      if (c >= 1) unpack(c - 1, 1);  // overlaps chunk c's reduce
      const auto t4 = clk::now();
      t_wait += secs(t0, t1), t_pack += secs(t1, t2), t_issue += secs(t2, t3), t_unpack += secs(t3, t4);
      continue;
    }
    // ONE H2D of the chunk's rows on the copy stream, once the reduce of chunk c-2 is done with d_stage[buf].
    // That reduce has normally finished long before (it is a few microseconds of a chunk's DMA time):
    // the copy queue is then not made to wait on the compute queue at all — a cross-queue wait in
    // front of every DMA stalls the copy engine between chunks.  DLA_HOST_WAIT_ALWAYS=1: always wait (A/B).
    if (c >= 2) {
      static const bool always = tuning_env("DLA_HOST_WAIT_ALWAYS") != nullptr;
      const hipError_t q = always ? hipErrorNotReady : hipEventQuery(red[buf]);
      if (q == hipErrorNotReady) {
        (void)hipGetLastError();
        if (!check(hipStreamWaitEvent(xs, red[buf], 0), "wait")) break;
      } else if (!check(q, "event query")) {
        break;
      }
    }
    if (!check(hipMemcpyAsync(ds, hs, static_cast<size_t>(rp * n_peers), hipMemcpyHostToDevice, xs), "H2D")) break;
    if (!check(hipEventRecord(h2d[buf], xs), "record")) break;
    // reduce (list order, fedavg.py:23-25) and D2H on the compute stream
    if (!check(hipStreamWaitEvent(cs_, h2d[buf], 0), "wait")) break;
    const int rc = wsum_impl(dtype, rows.data(), weights, n_peers, m, dout, stream, nullptr);
    if (rc != DLA_OK) {  // wsum_impl set the message; drain the copies still reading the caller's buffers
      (void)hipStreamSynchronize(cs_);
      (void)hipStreamSynchronize(xs);
      return rc;
    }
    if (!check(hipEventRecord(red[buf], cs_), "record")) break;
    if (!check(hipMemcpyAsync(hout, dout, m * es, hipMemcpyDeviceToHost, cs_), "D2H")) break;
    if (!check(hipEventRecord(d2h[buf], cs_), "record")) break;
    const auto t3 = clk::now();
    if (c >= 1) unpack(c - 1, 1);  // overlaps chunk c's H2D
    const auto t4 = clk::now();
    t_wait += secs(t0, t1), t_pack += secs(t1, t2), t_issue += secs(t2, t3), t_unpack += secs(t3, t4);
  }
  const auto t_loop = clk::now();
  if (e == hipSuccess) unpack(n_chunks - 1, 4);  // nothing left to overlap: spread it
  if (stats)
    std::fprintf(stderr,
                 "dla_host_reduce%s: %d peers x %lld elems, %lld chunks of <= %lld: total %.2f ms, first pack %.2f, "
                 "wait-h2d %.2f, pack %.2f (%.1f GB/s), issue %.2f, unpack+wait-d2h %.2f, last unpack %.2f\n",
                 mapped ? " (peers read in place)" : stage_read ? " (packed rows read in place)" : "", n_peers, static_cast<long long>(end - begin),
                 static_cast<long long>(n_chunks),
                 static_cast<long long>(chunk_elems), secs(t_start, clk::now()) * 1e3, t_first * 1e3, t_wait * 1e3,
                 t_pack * 1e3, t_pack > 0 ? double(end - begin) * es * n_peers / t_pack / 1e9 : 0.0, t_issue * 1e3,
                 t_unpack * 1e3, secs(t_loop, clk::now()) * 1e3);
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(cs_);
    (void)hipStreamSynchronize(xs);
    if (!outs_known && !g_last_error.empty()) return DLA_E_INVALID;  // abandoned / null outputs
    return static_cast<int>(e);
  }
  return DLA_OK;
}
}  // namespace

int64_t dla_host_in_place_rounds(void) { return g_host_in_place.load(std::memory_order_relaxed); }

int dla_host_reduce(int dtype, int n_peers, int n_tensors, const void* const* tensors, const int64_t* numels,
                    const double* weights, void* const* outs, int64_t begin, int64_t end, int64_t chunk_elems,
                    void* h_stage, void* d_stage, void* h_out, void* d_out, void* stream, void* copy_stream) {
  return host_reduce_impl(dtype, n_peers, n_tensors, tensors, numels, weights, outs, nullptr, begin, end, chunk_elems,
                          h_stage, d_stage, h_out, d_out, stream, copy_stream);
}

int dla_host_reduce_deferred(int dtype, int n_peers, int n_tensors, const void* const* tensors, const int64_t* numels,
                             const double* weights, void* const* outs, const int* outs_ready, int64_t begin,
                             int64_t end, int64_t chunk_elems, void* h_stage, void* d_stage, void* h_out, void* d_out,
                             void* stream, void* copy_stream) {
  if (!outs_ready) return fail(DLA_E_INVALID, "dla_host_reduce_deferred: outs_ready is required");
  return host_reduce_impl(dtype, n_peers, n_tensors, tensors, numels, weights, outs, outs_ready, begin, end,
                          chunk_elems, h_stage, d_stage, h_out, d_out, stream, copy_stream);
}

struct dla_host_job {
  std::thread th;  // only when no persistent worker was free (a concurrent launch on the same device)
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  int rc = DLA_OK;
  std::string err;
  std::vector<double> weights;  // the caller's array may be a temporary
  std::function<void()> body;
  std::chrono::steady_clock::time_point t_launch, t_start, t_end;
};

namespace {
// One persistent worker thread per HIP device runs launched host rounds: a new thread per round
// pays its creation and the HIP runtime's first-call set-up on that thread (hipSetDevice, event
// creation) on the round's critical path.  A worker holds at most one job; a launch that finds it
// busy (two rounds at once on one device) gets a thread of its own.  Rebuilt in a forked child,
// which has none of the parent's threads; never destroyed (the workers sleep until exit).
class HostWorkers {
 public:
  static HostWorkers& get() {
    static HostWorkers* w = new HostWorkers;  // leaked on purpose
    return *w;
  }
  bool try_post(int device, dla_host_job* j) {
    std::lock_guard<std::mutex> g(mu_);
    if (pid_ != getpid()) {  // forked: the parent's workers do not exist here
      slots_.clear();
      pid_ = getpid();
    }
    Slot* sl = slots_[device];
    if (!sl) {
      Slot* fresh = new Slot;  // leaked on purpose: no join at exit
      try {
        fresh->th = std::thread([fresh, device] { loop(fresh, device); });
      } catch (...) {
        delete fresh;  // no worker: this launch gets a thread of its own (or fails there)
        slots_.erase(device);
        return false;
      }
      fresh->th.detach();
      sl = slots_[device] = fresh;
    }
    std::lock_guard<std::mutex> sg(sl->mu);
    if (sl->job) return false;
    sl->job = j;
    sl->cv.notify_one();
    return true;
  }

 private:
  struct Slot {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    dla_host_job* job = nullptr;
  };
  static void loop(Slot* sl, int device) {
    (void)hipSetDevice(device);
    for (;;) {
      dla_host_job* j;
      {
        std::unique_lock<std::mutex> g(sl->mu);
        sl->cv.wait(g, [sl] { return sl->job != nullptr; });
        j = sl->job;
      }
      // run a copy: the joiner may free the job as soon as the body has signalled completion
      std::function<void()> body = std::move(j->body);
      body();
      {
        std::lock_guard<std::mutex> g(sl->mu);
        sl->job = nullptr;
      }
    }
  }
  std::mutex mu_;
  pid_t pid_ = getpid();
  std::map<int, Slot*> slots_;
};
}  // namespace

int dla_host_reduce_launch(int device, int dtype, int n_peers, int n_tensors, const void* const* tensors,
                           const int64_t* numels, const double* weights, void* const* outs, const int* outs_ready,
                           int64_t begin, int64_t end, int64_t chunk_elems, void* h_stage, void* d_stage, void* h_out,
                           void* d_out, void* stream, void* copy_stream, dla_host_job_t** job) {
  g_last_error.clear();
  if (!job) return fail(DLA_E_INVALID, "dla_host_reduce_launch: job is required");
  *job = nullptr;
  if (n_peers < 1 || !weights) return fail(DLA_E_INVALID, "dla_host_reduce_launch: need n_peers >= 1 and weights");
  int n_dev = 0;
  const hipError_t de = hipGetDeviceCount(&n_dev);
  if (de != hipSuccess || device < 0 || device >= n_dev)
    return fail(DLA_E_INVALID, "dla_host_reduce_launch: no HIP device " + std::to_string(device));
  dla_host_job* j = new (std::nothrow) dla_host_job;
  if (!j) return fail(DLA_E_INVALID, "dla_host_reduce_launch: out of memory");
  j->weights.assign(weights, weights + n_peers);
  j->t_launch = std::chrono::steady_clock::now();
  j->body = [=] {
    j->t_start = std::chrono::steady_clock::now();
    int rc;
    std::string err;
    const hipError_t se = hipSetDevice(device);
    if (se != hipSuccess) {
      rc = static_cast<int>(se);
      err = std::string("dla_host_reduce_launch: hipSetDevice: ") + hipGetErrorString(se);
    } else {
      rc = host_reduce_impl(dtype, n_peers, n_tensors, tensors, numels, j->weights.data(), outs, outs_ready, begin,
                            end, chunk_elems, h_stage, d_stage, h_out, d_out, stream, copy_stream);
      if (rc != DLA_OK) err = g_last_error;  // this worker thread's message
    }
    std::lock_guard<std::mutex> g(j->mu);
    j->rc = rc;
    j->err = err;
    j->t_end = std::chrono::steady_clock::now();
    j->done = true;
    j->cv.notify_all();
  };
  try {
    if (!HostWorkers::get().try_post(device, j)) j->th = std::thread(j->body);
  } catch (const std::exception& ex) {
    delete j;
    return fail(DLA_E_INVALID, std::string("dla_host_reduce_launch: ") + ex.what());
  }
  *job = j;
  return DLA_OK;
}

int dla_host_reduce_join(dla_host_job_t* job) {
  g_last_error.clear();
  if (!job) return fail(DLA_E_INVALID, "dla_host_reduce_join: null job");
  {
    std::unique_lock<std::mutex> g(job->mu);
    job->cv.wait(g, [job] { return job->done; });
  }
  if (job->th.joinable()) job->th.join();
  static const bool stats = tuning_env("DLA_HOST_REDUCE_STATS") != nullptr;
  if (stats) {
    const auto now = std::chrono::steady_clock::now();
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    std::fprintf(stderr, "dla_host_reduce_join: launch->start %.3f ms, run %.3f ms, end->join %.3f ms\n",
                 ms(job->t_launch, job->t_start), ms(job->t_start, job->t_end), ms(job->t_end, now));
  }
  const int rc = job->rc;
  if (rc != DLA_OK) g_last_error = job->err;
  delete job;
  return rc;
}

int dla_shard_range(int dtype, int64_t n_elems, int n_shards, int shard, int64_t* start, int64_t* end) {
  g_last_error.clear();
  const int es = elem_size(dtype);
  if (es == 0 || n_elems < 0 || n_shards < 1 || shard < 0 || shard >= n_shards || !start || !end)
    return fail(DLA_E_INVALID, "dla_shard_range: bad arguments");
  const int64_t per = shard_bucket_elems(es, n_elems, n_shards);
  *start = per * shard < n_elems ? per * shard : n_elems;
  *end = per * (shard + 1) < n_elems ? per * (shard + 1) : n_elems;
  return DLA_OK;
}

int dla_wsum_sharded(int dtype, int n_shards, const int* dev_ids, const void* const* peers, const double* weights,
                     int n_peers, int64_t n_elems, void* const* outs, int gather, void* const* streams) {
  return wsum_sharded_impl(dtype, n_shards, dev_ids, peers, weights, n_peers, n_elems, outs, gather, streams);
}

int dla_shutdown(void) {
  g_last_error.clear();
  std::lock_guard<std::mutex> lock(g_shard_mu);
  DeviceGuard guard;
  for (auto& de : g_event_pool) {
    if (hipSetDevice(de.first) == hipSuccess) (void)hipEventDestroy(de.second);
  }
  g_event_pool.clear();
  for (auto& ds : g_table_streams) {
    if (hipSetDevice(ds.first) == hipSuccess) (void)hipStreamDestroy(ds.second);
  }
  g_table_streams.clear();
  for (const auto& pr : g_peer_enabled) {
    if (hipSetDevice(pr.first) == hipSuccess) (void)hipDeviceDisablePeerAccess(pr.second);
  }
  g_peer_enabled.clear();
  (void)hipGetLastError();
  return DLA_OK;
}

int dla_wsum_slab_tiled(int dtype, const void* base, int64_t tile_elems, int64_t slab_rows, const double* weights,
                        int n_peers, int64_t n_elems, void* out, void* stream, const dla_launch_cfg_t* cfg) {
  g_last_error.clear();
  const int es = elem_size(dtype);
  if (es == 0 || dtype == DLA_F64)
    return fail(DLA_E_INVALID, "dla_wsum_slab_tiled: dtype must be F32, BF16 or F16");
  if (!base || !weights || n_peers < 1 || n_peers > slab_rows || n_elems < 0)
    return fail(DLA_E_INVALID, "dla_wsum_slab_tiled: need base, weights and 1 <= n_peers <= slab_rows");
  if (tile_elems < 1 || (tile_elems & (tile_elems - 1)) || tile_elems * es < 16)
    return fail(DLA_E_INVALID, "dla_wsum_slab_tiled: tile_elems must be a power of two of >= 16 bytes");
  if ((reinterpret_cast<uintptr_t>(base) & 15u) || (reinterpret_cast<uintptr_t>(out) & 15u))
    return fail(DLA_E_INVALID, "dla_wsum_slab_tiled: base and out must be 16-byte aligned");
  if (n_elems == 0) return DLA_OK;
  if (!out) return fail(DLA_E_INVALID, "dla_wsum_slab_tiled: null out");
  int tshift = 0;
  while ((int64_t{1} << tshift) < tile_elems) ++tshift;
  const int first_pass = n_peers < kMaxPeersPerPass ? n_peers : kMaxPeersPerPass;
  int variant = cfg && cfg->variant ? cfg->variant : vec_store_policy(vec_variant(first_pass), n_elems * es);
  if (!(cfg && cfg->variant) && first_pass >= 32 && int64_t{first_pass} * n_elems * es >= (int64_t{1} << 30))
    variant = first_pass == 64 ? 8 : 12;  // fewer peers per round under the occupancy cap (vec_wgs_cap)
  if (variant != 8 && variant != 9 && variant != 12 && variant != 21 && variant != 28)
    return fail(DLA_E_CONFIG, "dla_wsum_slab_tiled: variant must be 0 (auto), 8, 9, 12, 21 or 28");
  const int64_t stride = slab_rows * tile_elems;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e;
  switch (dtype) {
    case DLA_F32: e = run_tiled<DLA_F32>(base, tile_elems, tshift, stride, weights, n_peers, n_elems, out, s, variant); break;
    case DLA_BF16: e = run_tiled<DLA_BF16>(base, tile_elems, tshift, stride, weights, n_peers, n_elems, out, s, variant); break;
    default: e = run_tiled<DLA_F16>(base, tile_elems, tshift, stride, weights, n_peers, n_elems, out, s, variant); break;
  }
  if (e != hipSuccess) return fail(static_cast<int>(e), std::string("dla_wsum_slab_tiled: ") + hipGetErrorString(e));
  return DLA_OK;
}

int dla_slab_stage(int dtype, void* base, int64_t tile_elems, int64_t slab_rows, int64_t n_tiles, int row,
                   int64_t dst_elem, const void* src, int64_t n_elems, void* stream) {
  g_last_error.clear();
  const int es = elem_size(dtype);
  if (es == 0) return fail(DLA_E_INVALID, "dla_slab_stage: unknown dtype");
  if (!base || tile_elems < 1 || slab_rows < 1 || row < 0 || row >= slab_rows || dst_elem < 0 || n_elems < 0)
    return fail(DLA_E_INVALID, "dla_slab_stage: need base, tile_elems >= 1 and 0 <= row < slab_rows");
  // the range must lie inside the slab's row: a bad argument fails here instead of letting the copy
  // engine write past the end of the HBM buffer
  if (n_tiles < 0 || n_tiles > (INT64_MAX / tile_elems) || dst_elem > n_tiles * tile_elems ||
      n_elems > n_tiles * tile_elems - dst_elem)
    return fail(DLA_E_INVALID, "dla_slab_stage: elements [" + std::to_string(dst_elem) + ", " +
                                   std::to_string(dst_elem + n_elems) + ") do not fit the row's " +
                                   std::to_string(n_tiles) + " tiles of " + std::to_string(tile_elems));
  if (n_elems == 0) return DLA_OK;
  if (!src) return fail(DLA_E_INVALID, "dla_slab_stage: null src");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t tb = tile_elems * es;  // bytes of one tile
  char* b = static_cast<char*>(base);
  const char* p = static_cast<const char*>(src);
  int64_t pos = dst_elem, left = n_elems;
  // element pos of the row lives at tile pos / tile_elems, slab row `row`, offset pos % tile_elems
  auto at = [&](int64_t e) { return b + (((e / tile_elems) * slab_rows + row) * tile_elems + e % tile_elems) * es; };
  auto failed = [](hipError_t e, const char* what) {
    return fail(static_cast<int>(e), std::string("dla_slab_stage: ") + what + ": " + hipGetErrorString(e));
  };
  hipError_t e;
  if (pos % tile_elems) {  // the partial tile the range starts in
    const int64_t m = std::min(tile_elems - pos % tile_elems, left);
    if ((e = hipMemcpyAsync(at(pos), p, static_cast<size_t>(m * es), hipMemcpyDefault, s)) != hipSuccess)
      return failed(e, "head");
    pos += m, left -= m, p += m * es;
  }
  const int64_t full = left / tile_elems;
  if (full) {  // every whole tile in one 2D copy: rows of one tile, destination pitch = slab_rows tiles
    if ((e = hipMemcpy2DAsync(at(pos), static_cast<size_t>(slab_rows * tb), p, static_cast<size_t>(tb),
                              static_cast<size_t>(tb), static_cast<size_t>(full), hipMemcpyDefault, s)) != hipSuccess)
      return failed(e, "tiles");
    pos += full * tile_elems, left -= full * tile_elems, p += full * tb;
  }
  if (left && (e = hipMemcpyAsync(at(pos), p, static_cast<size_t>(left * es), hipMemcpyDefault, s)) != hipSuccess)
    return failed(e, "tail");
  return DLA_OK;
}

int64_t dla_slab_tile_elems(int dtype, int slab_rows, int64_t n_elems) {
  const int es = elem_size(dtype);
  if (es == 0 || slab_rows < 1 || n_elems < 0) return 0;
  // Interleaved A/B over tile sizes 1, 4 and 16 KiB (profiles/r02d_ab_tiled.log): 16 KiB for up to
  // 16 rows (8 x 25 M f32 130.2 / 131.1 / 132.1 us for 16 / 4 / 1 KiB; 16 x 21.3 M bf16 106.3 /
  // 108.3 / 109.2), 1 KiB for rows under 1 MiB (128 x 85 354 f32 9.5 / 10.9 / 9.8), else 4 KiB
  // (128 x 21.3 M bf16 792 / 796 / 831; 64 x 1.23 M f32 47.5 / 55.2 / 48.5; within 2 % of the
  // best elsewhere: 128 x 2.66 M bf16 103.6 vs 102.7, 32 x 1.69 M f32 33.5 vs 32.8).  Under the
  // occupancy cap (round 3) 32 KiB tiles for up to 8 rows: 8 x 25 M f32 125.2-125.5 us against
  // 125.8-126.0 for 16 KiB, 128.4-128.7 for 64 KiB, 129.8-130.2 for 4 KiB (profiles/r03ak, r03al).
  int64_t bytes = 4096;
  if (n_elems * es < (int64_t{1} << 20))
    bytes = 1024;
  else if (slab_rows <= 8)
    bytes = 32768;
  else if (slab_rows <= 16)
    bytes = 16384;
  return bytes / es;
}

}  // extern "C"
