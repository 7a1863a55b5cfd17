// probe.hip — HBM ceiling probes for MI355X (diagnostics, not on the product path).
//
// bench.py --sweep times these beside the FedAvg kernel so the roofline fraction can
// be read against what this chip actually streams (measured ceilings), not only
// against the 8 TB/s datasheet number:
//   dlp_read  — every lane streams 16-byte chunks (CH per lane, all issued before the
//               first use), XOR-folds them; one dword per workgroup is written only if
//               the fold hits a magic value (never), so the loads cannot be removed.
//   dlp_copy  — dwordx4 copy (read + write, 1:1).
#include <hip/hip_runtime.h>

#include <cstdint>

// Hash of this file and the compile flags, set by the build (accdfl_amd/_lib.py build_probe()): a
// probe library is rebuilt when its id differs from the tree's, not by file times.
#ifndef DLP_BUILD_ID
#define DLP_BUILD_ID "unversioned"
#endif

namespace {

__attribute__((used)) const char kProbeIdTag[] = "dlagg-probe-build-id:" DLP_BUILD_ID;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int CH, bool NT>
__global__ __launch_bounds__(256) void read_kernel(const u32x4* __restrict__ src, int64_t n_chunks,
                                                    uint32_t* __restrict__ sink) {
  const int64_t base = static_cast<int64_t>(blockIdx.x) * 256 * CH + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 v[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    int64_t i = base + c * 256;
    i = i < n_chunks ? i : n_chunks - 1;
    v[c] = NT ? __builtin_nontemporal_load(src + i) : src[i];
  }
#pragma unroll
  for (int c = 0; c < CH; ++c) acc ^= v[c];
  const uint32_t f = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (f == 0x9e3779b9u && threadIdx.x == 0) sink[blockIdx.x & 1023] = f;
}

template <int CH, bool NT>
__global__ __launch_bounds__(256) void copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                    int64_t n_chunks) {
  const int64_t base = static_cast<int64_t>(blockIdx.x) * 256 * CH + threadIdx.x;
  u32x4 v[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int64_t i = base + c * 256;
    if (i < n_chunks) v[c] = NT ? __builtin_nontemporal_load(src + i) : src[i];
  }
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int64_t i = base + c * 256;
    if (i < n_chunks) dst[i] = v[c];
  }
}

// Peer-major "big tile" FedAvg probe (f32, 8 peers): one wave owns 64*CH contiguous
// chunks (CH*1 KiB of output); it streams peer 0's CH chunks, then peer 1's, ... (the loads
// of peer k+1 are in flight while peer k is folded), then writes its CH chunks.  With a
// persistent grid the chip reads in long phases and writes in short bursts, instead of
// mixing 8 reads and 1 write at every tile.  Same per-element fold order as the product.
template <int CH, int PF>
__global__ __launch_bounds__(64) void bigtile_kernel(const u32x4* s0, const u32x4* s1, const u32x4* s2,
                                                     const u32x4* s3, const u32x4* s4, const u32x4* s5,
                                                     const u32x4* s6, const u32x4* s7, float w0, float w1,
                                                     float w2, float w3, float w4, float w5, float w6, float w7,
                                                     int64_t n_chunks, u32x4* __restrict__ dst) {
  const u32x4* src[8] = {s0, s1, s2, s3, s4, s5, s6, s7};
  const float w[8] = {w0, w1, w2, w3, w4, w5, w6, w7};
  const int64_t n_big = n_chunks / (64 * CH);  // full big tiles only (the probe ignores the rest)
  for (int64_t big = blockIdx.x; big < n_big; big += gridDim.x) {
    const int64_t base = big * 64 * CH + threadIdx.x;
    float acc[CH][4];
    u32x4 a[CH], b[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = __builtin_nontemporal_load(src[0] + base + c * 64);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (PF == 2 && k + 1 < 8) {
#pragma unroll
        for (int c = 0; c < CH; ++c) b[c] = __builtin_nontemporal_load(src[k + 1] + base + c * 64);
      }
      asm volatile("" ::: "memory");  // keep peer k+2's loads below peer k's fold (two buffers)
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const float x[4] = {__uint_as_float(a[c].x), __uint_as_float(a[c].y), __uint_as_float(a[c].z),
                            __uint_as_float(a[c].w)};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (k == 0) acc[c][e] = x[e] * 0.0f;
          acc[c][e] = acc[c][e] + w[k] * x[e];
        }
      }
      if constexpr (PF == 2) {
#pragma unroll
        for (int c = 0; c < CH; ++c) a[c] = b[c];
      } else if (k + 1 < 8) {  // one buffer: the next peer's loads issue after this fold
#pragma unroll
        for (int c = 0; c < CH; ++c) a[c] = __builtin_nontemporal_load(src[k + 1] + base + c * 64);
      }
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const u32x4 v = {__float_as_uint(acc[c][0]), __float_as_uint(acc[c][1]), __float_as_uint(acc[c][2]),
                       __float_as_uint(acc[c][3])};
      asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst + base + c * 64), "v"(v) : "memory");
    }
  }
}

// Pure write stream: every lane stores CH 16-byte chunks of a constant (SC1: sc1 stores).
template <int CH, bool SC1>
__global__ __launch_bounds__(256) void write_kernel(u32x4* __restrict__ dst, int64_t n_chunks, uint32_t val) {
  const int64_t base = static_cast<int64_t>(blockIdx.x) * 256 * CH + threadIdx.x;
  const u32x4 v = {val, val ^ 1u, val ^ 2u, val ^ 3u};
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int64_t i = base + c * 256;
    if (i < n_chunks) {
      if constexpr (SC1)
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst + i), "v"(v) : "memory");
      else
        dst[i] = v;
    }
  }
}

// The FedAvg access pattern without the arithmetic: each lane loads the same 16-byte
// chunk offset from N_SRC separate buffers (all issued first), folds them, and
// (WRITE) stores the fold to dst — isolates multi-stream reads vs the output write.
template <int N_SRC, int CH, bool WRITE>
__global__ __launch_bounds__(256) void mread_kernel(const u32x4* const* __restrict__ srcs_unused,
                                                     const u32x4* s0, const u32x4* s1, const u32x4* s2,
                                                     const u32x4* s3, const u32x4* s4, const u32x4* s5,
                                                     const u32x4* s6, const u32x4* s7, int64_t n_chunks,
                                                     u32x4* __restrict__ dst, uint32_t* __restrict__ sink,
                                                     int sc1) {
  const u32x4* src[8] = {s0, s1, s2, s3, s4, s5, s6, s7};
  const int64_t base = static_cast<int64_t>(blockIdx.x) * 256 * CH + threadIdx.x;
  int64_t idx[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int64_t i = base + c * 256;
    idx[c] = i < n_chunks ? i : n_chunks - 1;
  }
  u32x4 v[N_SRC][CH];
#pragma unroll
  for (int k = 0; k < N_SRC; ++k)
#pragma unroll
    for (int c = 0; c < CH; ++c) v[k][c] = __builtin_nontemporal_load(src[k] + idx[c]);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    u32x4 acc = v[0][c];
#pragma unroll
    for (int k = 1; k < N_SRC; ++k) acc ^= v[k][c];
    if constexpr (WRITE) {
      if (base + c * 256 < n_chunks) {
        if (sc1)
          asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst + idx[c]), "v"(acc) : "memory");
        else
          dst[idx[c]] = acc;
      }
    } else {
      const uint32_t f = acc.x ^ acc.y ^ acc.z ^ acc.w;
      if (f == 0x9e3779b9u) sink[blockIdx.x & 1023] = f;
    }
  }
}

template <int CH>
int launch_read(const void* src, int64_t bytes, void* sink, int nt, hipStream_t s) {
  const int64_t n = bytes / 16;
  const int64_t grid = (n + 256 * CH - 1) / (256 * CH);
  if (nt)
    hipLaunchKernelGGL((read_kernel<CH, true>), dim3(grid), dim3(256), 0, s, static_cast<const u32x4*>(src), n,
                       static_cast<uint32_t*>(sink));
  else
    hipLaunchKernelGGL((read_kernel<CH, false>), dim3(grid), dim3(256), 0, s, static_cast<const u32x4*>(src), n,
                       static_cast<uint32_t*>(sink));
  return static_cast<int>(hipGetLastError());
}

// Tile-interleaved layout probe: peers stored as [tiles][NS][T chunks] (T = 64 * CH,
// one wave per workgroup), so a workgroup reads one contiguous NS*T*16-byte region.
// OUT_SLOT: the output goes to slot NS of a [tiles][NS+1][T] layout (same region) instead
// of a separate flat buffer.
template <int NS, int CH, bool OUT_SLOT>
__global__ __launch_bounds__(64) void tiled_kernel(const u32x4* __restrict__ src, int64_t n_tiles,
                                                    u32x4* __restrict__ dst) {
  constexpr int T = 64 * CH;
  const int64_t tile = blockIdx.x;
  if (tile >= n_tiles) return;
  constexpr int SLOTS = OUT_SLOT ? NS + 1 : NS;
  const u32x4* base = src + tile * SLOTS * T;
  u32x4 v[NS][CH];
#pragma unroll
  for (int k = 0; k < NS; ++k)
#pragma unroll
    for (int c = 0; c < CH; ++c) v[k][c] = __builtin_nontemporal_load(base + k * T + c * 64 + threadIdx.x);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    u32x4 acc = v[0][c];
#pragma unroll
    for (int k = 1; k < NS; ++k) acc ^= v[k][c];
    u32x4* o = OUT_SLOT ? const_cast<u32x4*>(base) + NS * T + c * 64 + threadIdx.x : dst + tile * T + c * 64 + threadIdx.x;
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(o), "v"(acc) : "memory");
  }
}

// Load cache-policy probe on the FedAvg pattern (8 streams + 1 sc1 write, 64-thread WGs,
// 1 chunk/lane).  POL: 0 "nt" (compiler builtin), 1 "sc1", 2 "sc0 sc1", 3 "sc0 sc1 nt", 4 "sc1 nt".
// The asm loads are waited by an asm that takes every loaded register as "+v", so no use
// can be scheduled before the wait.
#define DLP_LD(POLSTR, dst, ptr) asm volatile("global_load_dwordx4 %0, %1, off " POLSTR : "=v"(dst) : "v"(ptr) : "memory")
template <int POL>
__global__ __launch_bounds__(64) void policy_kernel(const u32x4* s0, const u32x4* s1, const u32x4* s2,
                                                     const u32x4* s3, const u32x4* s4, const u32x4* s5,
                                                     const u32x4* s6, const u32x4* s7, int64_t n_chunks,
                                                     u32x4* __restrict__ dst) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 64 + threadIdx.x;
  if (i >= n_chunks) return;
  const u32x4* src[8] = {s0, s1, s2, s3, s4, s5, s6, s7};
  u32x4 v[8];
  if constexpr (POL == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(src[k] + i);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const u32x4* a = src[k] + i;
      if constexpr (POL == 1) DLP_LD("sc1", v[k], a);
      if constexpr (POL == 2) DLP_LD("sc0 sc1", v[k], a);
      if constexpr (POL == 3) DLP_LD("sc0 sc1 nt", v[k], a);
      if constexpr (POL == 4) DLP_LD("sc1 nt", v[k], a);
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]),
                 "+v"(v[6]), "+v"(v[7])::"memory");
  }
  u32x4 acc = v[0];
#pragma unroll
  for (int k = 1; k < 8; ++k) acc ^= v[k];
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst + i), "v"(acc) : "memory");
}
#undef DLP_LD

// Width-calibration read: each lane reads W bytes (4, 8 or 16) per load, 4 loads in flight per
// lane, nt.  Over a buffer of known size this calibrates rocprofv3's FETCH_SIZE for the load
// width the word-per-lane FedAvg kernels use (MI355X_MICROARCH.md: only 16-B reads are calibrated).
template <typename V>
__global__ __launch_bounds__(256) void read_w_kernel(const V* __restrict__ src, int64_t n, uint32_t* __restrict__ sink) {
  const int64_t base = static_cast<int64_t>(blockIdx.x) * 1024 + threadIdx.x;
  V v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    int64_t i = base + c * 256;
    i = i < n ? i : n - 1;
    v[c] = __builtin_nontemporal_load(src + i);
  }
  uint32_t f = 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(&v[c]);
#pragma unroll
    for (int d = 0; d < static_cast<int>(sizeof(V) / 4); ++d) f ^= q[d];
  }
  if (f == 0x9e3779b9u && threadIdx.x == 0) sink[blockIdx.x & 1023] = f;
}

// The many-peer access pattern of the word-per-lane FedAvg kernels without the arithmetic:
// lane j of workgroup b reads vector (b * 64 + j) of each of n_src rows (W bytes per lane), G rows
// at a time, XOR-folded; one W-byte output per lane written sc1 (write=1) or nothing.
struct SrcTable { const void* p[128]; };
template <typename V, int G, bool WRITE>
__global__ __launch_bounds__(64) void mread_w_kernel(const SrcTable tab, int n_src, int64_t n, V* __restrict__ dst,
                                                     uint32_t* __restrict__ sink) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * 64 + threadIdx.x;
  const int64_t i = j < n ? j : n - 1;
  V acc;
  __builtin_memset(&acc, 0, sizeof(V));
  for (int k0 = 0; k0 < n_src; k0 += G) {
    V v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int k = k0 + g < n_src ? k0 + g : n_src - 1;
      v[g] = __builtin_nontemporal_load(static_cast<const V*>(tab.p[k]) + i);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) acc ^= v[g];
  }
  if constexpr (WRITE) {
    if (j < n) dst[j] = acc;
  } else {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(&acc);
    if (q[0] == 0x9e3779b9u) sink[blockIdx.x & 1023] = q[0];
  }
}

// As mread_w_kernel with the rounds over the 128-row table unrolled (compile-time table
// indices, as wsum_vec_kernel): the FedAvg kernel's exact load / store schedule, XOR in place
// of the fold.  Tile-interleaved layout when tile_vecs > 0: vector i of row k lives at
// base_k + (i / tile_vecs) * stride_vecs + i % tile_vecs.
template <typename V, int G, bool WRITE>
__global__ __launch_bounds__(64) void mread_unrolled_kernel(const SrcTable tab, int64_t n, V* __restrict__ dst,
                                                            uint32_t* __restrict__ sink, int64_t tile_vecs,
                                                            int64_t stride_vecs) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * 64 + threadIdx.x;
  const int64_t i = j < n ? j : n - 1;
  const int64_t a = tile_vecs > 0 ? (i / tile_vecs) * stride_vecs + i % tile_vecs : i;
  V acc;
  __builtin_memset(&acc, 0, sizeof(V));
#pragma unroll
  for (int r = 0; r < 128 / G; ++r) {
    V v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) v[g] = __builtin_nontemporal_load(static_cast<const V*>(tab.p[r * G + g]) + a);
#pragma unroll
    for (int g = 0; g < G; ++g) acc ^= v[g];
  }
  if constexpr (WRITE) {
    if (j < n) dst[j] = acc;
  } else {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(&acc);
    if (q[0] == 0x9e3779b9u) sink[blockIdx.x & 1023] = q[0];
  }
}

// LDS-DMA staging of the north star: the FedAvg fp32 fold of 8 peers held in
// the tile-interleaved slab ([tiles][8][4096 f32], 16 KiB tiles — the headline's layout), with
// every peer load a global_load_lds_dwordx4 into LDS instead of a VGPR load.  Persistent: a
// one-wave workgroup walks units u = wave, wave + n_waves, ... of 1 KiB of output (64 lanes x
// 16 B) through S LDS stages of 8 x 1 KiB, so S x 8 KiB per wave are in flight with no VGPR
// held for them.  A stage is consumed after `s_waitcnt vmcnt(8 (S - 1))` — the loads of the S - 1
// younger stages may stay in flight; the output stores, if the counter tallies them, only make
// that wait stricter.  Each lane reads back only the 16 B it loaded (an LDS-DMA piece lands at
// base + lane x 16), so the issuing wave's own counter is the only ordering needed.  The fold is
// the product's fp32 fold (p0 * 0, then acc + w * p in list order, no FMA), so the probe's output
// is compared bit for bit with dla_wsum_slab_tiled's.  Units past n_units (the < 256-element
// tail) are not computed.
template <int S>
__global__ __launch_bounds__(64) void ldsdma_tiled8_kernel(const float* __restrict__ slab, const float w0,
                                                           const float w1, const float w2, const float w3,
                                                           const float w4, const float w5, const float w6,
                                                           const float w7, int64_t n_units, float* __restrict__ out) {
  __shared__ u32x4 stage[S][8][64];
  const float w[8] = {w0, w1, w2, w3, w4, w5, w6, w7};
  const int lane = threadIdx.x;
  const int64_t n_waves = gridDim.x;
  const int64_t first = blockIdx.x;
  // unit u: tile u >> 4, 1 KiB piece u & 15 of it; peer k's piece at ((u >> 4) * 8 + k) * 4096 + (u & 15) * 256
  auto issue = [&](int b, int64_t u) {
    const float* src = slab + ((u >> 4) * 8) * 4096 + (u & 15) * 256 + lane * 4;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t lds = __builtin_amdgcn_readfirstlane(
          static_cast<uint32_t>(reinterpret_cast<uintptr_t>(&stage[b][k][0])));
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(src + k * 4096), "s"(lds) : "memory");
    }
  };
  int64_t u = first;
#pragma unroll
  for (int b = 0; b < S; ++b)
    if (u + b * n_waves < n_units) issue(b, u + b * n_waves);
  if (u + (S - 1) * n_waves >= n_units) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // < S stages issued
  for (int it = 0; u < n_units; ++it, u += n_waves) {
    const int b = it % S;
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * (S - 1)) : "memory");
    u32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = stage[b][k][lane];
    float acc[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] = __uint_as_float(v[0][e]) * 0.0f;  // fedavg.py:22
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = acc[e] + w[k] * __uint_as_float(v[k][e]);  // fedavg.py:25
    u32x4 o = {__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]), __float_as_uint(acc[3])};
    u32x4* dst = reinterpret_cast<u32x4*>(out + u * 256) + lane;
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst), "v"(o) : "memory");
    const int64_t nu = u + S * n_waves;
    if (nu < n_units) {
      issue(b, nu);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain: the count above assumes S stages in flight
    }
  }
}

}  // namespace

extern "C" {

int dlp_policy8(const void* const* srcs, int64_t bytes_each, void* dst, int pol, void* stream) {
  if (!srcs || bytes_each < 16) return -1;
  const int64_t n = bytes_each / 16;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const u32x4* p[8];
  for (int k = 0; k < 8; ++k) p[k] = static_cast<const u32x4*>(srcs[k]);
  const dim3 g((n + 63) / 64);
#define DLP_P(POL) hipLaunchKernelGGL((policy_kernel<POL>), g, dim3(64), 0, s, p[0], p[1], p[2], p[3], p[4], p[5], \
                                      p[6], p[7], n, static_cast<u32x4*>(dst))
  switch (pol) {
    case 0: DLP_P(0); break;
    case 1: DLP_P(1); break;
    case 2: DLP_P(2); break;
    case 3: DLP_P(3); break;
    case 4: DLP_P(4); break;
    default: return -1;
  }
#undef DLP_P
  return static_cast<int>(hipGetLastError());
}


// bytes_each per peer (8 peers); layout [tiles][8 or 9][64*chunks*16 B]; out_slot 0/1.
int dlp_tiled8(void* slab, int64_t bytes_each, void* dst, int chunks, int out_slot, void* stream) {
  if (!slab || bytes_each < 16) return -1;
  const int64_t T = 64 * chunks;
  const int64_t n_tiles = bytes_each / 16 / T;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const u32x4* src = static_cast<const u32x4*>(slab);
  u32x4* d = static_cast<u32x4*>(dst);
#define DLP_T(CHV, OS) hipLaunchKernelGGL((tiled_kernel<8, CHV, OS>), dim3(n_tiles), dim3(64), 0, s, src, n_tiles, d)
  if (chunks == 1) { if (out_slot) DLP_T(1, true); else DLP_T(1, false); }
  else if (chunks == 4) { if (out_slot) DLP_T(4, true); else DLP_T(4, false); }
  else if (chunks == 16) { if (out_slot) DLP_T(16, true); else DLP_T(16, false); }
  else return -1;
#undef DLP_T
  return static_cast<int>(hipGetLastError());
}


// Read `bytes` (multiple of 16) from src; `chunks` in {1, 4, 8}; sink >= 4 KiB.
int dlp_read(const void* src, int64_t bytes, void* sink, int chunks, int nt, void* stream) {
  if (!src || !sink || bytes < 16) return -1;
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (chunks) {
    case 1: return launch_read<1>(src, bytes, sink, nt, s);
    case 4: return launch_read<4>(src, bytes, sink, nt, s);
    case 8: return launch_read<8>(src, bytes, sink, nt, s);
    default: return -1;
  }
}

// Copy `bytes` (multiple of 16) src -> dst with 4 chunks per lane.
int dlp_copy(const void* src, void* dst, int64_t bytes, int nt, void* stream) {
  if (!src || !dst || bytes < 16) return -1;
  const int64_t n = bytes / 16;
  const int64_t grid = (n + 1023) / 1024;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (nt)
    hipLaunchKernelGGL((copy_kernel<4, true>), dim3(grid), dim3(256), 0, s, static_cast<const u32x4*>(src),
                       static_cast<u32x4*>(dst), n);
  else
    hipLaunchKernelGGL((copy_kernel<4, false>), dim3(grid), dim3(256), 0, s, static_cast<const u32x4*>(src),
                       static_cast<u32x4*>(dst), n);
  return static_cast<int>(hipGetLastError());
}

// bigtile_kernel over 8 peers of bytes_each; chunks in {4, 8, 16}; grid 0 = one WG per big tile.
int dlp_bigtile8(const void* const* srcs, const float* w, int64_t bytes_each, void* dst, int chunks, int grid,
                 void* stream) {
  if (!srcs || !w || bytes_each < 16) return -1;
  const int64_t n = bytes_each / 16;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const u32x4* p[8];
  for (int k = 0; k < 8; ++k) p[k] = static_cast<const u32x4*>(srcs[k]);
#define DLP_B(CHV, PFV)                                                                                     \
  do {                                                                                                      \
    const int64_t nb = n / (64 * CHV);                                                     \
    const int64_t g = grid > 0 && grid < nb ? grid : nb;                                                    \
    hipLaunchKernelGGL((bigtile_kernel<CHV, PFV>), dim3(g), dim3(64), 0, s, p[0], p[1], p[2], p[3], p[4], p[5],  \
                       p[6], p[7], w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], n,                       \
                       static_cast<u32x4*>(dst));                                                           \
  } while (0)
  // chunks: 4, 8, 16, 24, 32 two peers in flight; 116, 124, 132 (100 + CH) one peer in flight
  if (chunks == 4) DLP_B(4, 2);
  else if (chunks == 8) DLP_B(8, 2);
  else if (chunks == 12) DLP_B(12, 2);
  else if (chunks == 16) DLP_B(16, 2);
  else if (chunks == 20) DLP_B(20, 2);
  else if (chunks == 120) DLP_B(20, 1);
  else if (chunks == 24) DLP_B(24, 2);
  else if (chunks == 32) DLP_B(32, 2);
  else if (chunks == 116) DLP_B(16, 1);
  else if (chunks == 124) DLP_B(24, 1);
  else if (chunks == 132) DLP_B(32, 1);
  else return -1;
#undef DLP_B
  return static_cast<int>(hipGetLastError());
}

// Write `bytes` (multiple of 16) of a constant; sc1 = 1 for sc1 stores.
int dlp_write(void* dst, int64_t bytes, int sc1, void* stream) {
  if (!dst || bytes < 16) return -1;
  const int64_t n = bytes / 16;
  const int64_t grid = (n + 1023) / 1024;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (sc1)
    hipLaunchKernelGGL((write_kernel<4, true>), dim3(grid), dim3(256), 0, s, static_cast<u32x4*>(dst), n, 0x3f800000u);
  else
    hipLaunchKernelGGL((write_kernel<4, false>), dim3(grid), dim3(256), 0, s, static_cast<u32x4*>(dst), n, 0x3f800000u);
  return static_cast<int>(hipGetLastError());
}

// 8-stream read (write = 0), read + write (write = 1) or read + sc1 write (write = 2).
int dlp_mread8(const void* const* srcs, int64_t bytes_each, void* dst, void* sink, int chunks, int write,
               void* stream) {
  if (!srcs || bytes_each < 16) return -1;
  const int64_t n = bytes_each / 16;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const u32x4* p[8];
  for (int k = 0; k < 8; ++k) p[k] = static_cast<const u32x4*>(srcs[k]);
#define DLP_L(CHV, W)                                                                                       \
  hipLaunchKernelGGL((mread_kernel<8, CHV, W>), dim3((n + 256 * CHV - 1) / (256 * CHV)), dim3(256), 0, s,   \
                     nullptr, p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], n, static_cast<u32x4*>(dst), \
                     static_cast<uint32_t*>(sink), write == 2)
  if (chunks == 1) { if (write) DLP_L(1, true); else DLP_L(1, false); }
  else if (chunks == 2) { if (write) DLP_L(2, true); else DLP_L(2, false); }
  else if (chunks == 4) { if (write) DLP_L(4, true); else DLP_L(4, false); }
  else return -1;
#undef DLP_L
  return static_cast<int>(hipGetLastError());
}

// Read `bytes` with `width` (4, 8 or 16) bytes per lane per load (FETCH_SIZE width calibration).
int dlp_read_width(const void* src, int64_t bytes, void* sink, int width, void* stream) {
  if (!src || !sink || bytes < 16) return -1;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n = bytes / width;
  const dim3 g(static_cast<unsigned>((n + 1023) / 1024)), b(256);
  uint32_t* sk = static_cast<uint32_t*>(sink);
  switch (width) {
    case 4: hipLaunchKernelGGL((read_w_kernel<uint32_t>), g, b, 0, s, static_cast<const uint32_t*>(src), n, sk); break;
    case 8: hipLaunchKernelGGL((read_w_kernel<u32x2>), g, b, 0, s, static_cast<const u32x2*>(src), n, sk); break;
    case 16: hipLaunchKernelGGL((read_w_kernel<u32x4>), g, b, 0, s, static_cast<const u32x4*>(src), n, sk); break;
    default: return -1;
  }
  return static_cast<int>(hipGetLastError());
}

// n_src (<= 128) rows of bytes_each, read `width` bytes per lane, `group` rows in flight per
// lane (16, 32 or 64 for width 4; 16 or 32 for 8; 8 or 16 for 16); write=1 also writes one row.
int dlp_mread_width(const void* const* srcs, int n_src, int64_t bytes_each, void* dst, void* sink, int width,
                    int group, int write, void* stream) {
  if (!srcs || n_src < 1 || n_src > 128 || !sink || bytes_each < 16) return -1;
  SrcTable t;
  for (int k = 0; k < 128; ++k) t.p[k] = srcs[k < n_src ? k : n_src - 1];
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n = bytes_each / width;
  const dim3 g(static_cast<unsigned>((n + 63) / 64)), b(64);
  uint32_t* sk = static_cast<uint32_t*>(sink);
#define DLP_MW(V, G)                                                                                       \
  do {                                                                                                     \
    if (write)                                                                                             \
      hipLaunchKernelGGL((mread_w_kernel<V, G, true>), g, b, 0, s, t, n_src, n, static_cast<V*>(dst), sk); \
    else                                                                                                   \
      hipLaunchKernelGGL((mread_w_kernel<V, G, false>), g, b, 0, s, t, n_src, n, static_cast<V*>(dst), sk); \
  } while (0)
  if (width == 4 && group == 16) DLP_MW(uint32_t, 16);
  else if (width == 4 && group == 32) DLP_MW(uint32_t, 32);
  else if (width == 4 && group == 64) DLP_MW(uint32_t, 64);
  else if (width == 8 && group == 16) DLP_MW(u32x2, 16);
  else if (width == 8 && group == 32) DLP_MW(u32x2, 32);
  else if (width == 16 && group == 8) DLP_MW(u32x4, 8);
  else if (width == 16 && group == 16) DLP_MW(u32x4, 16);
  else return -1;
#undef DLP_MW
  return static_cast<int>(hipGetLastError());
}

// The unrolled 128-row read (mread_unrolled_kernel): width 8 with group 16 or 32, width 16 with
// group 16; tile_bytes > 0 reads the tile-interleaved layout (row k's tile t at
// base + (t * 128 + k) * tile_bytes, srcs[k] = base + k * tile_bytes).
int dlp_mread_unrolled(const void* const* srcs, int64_t bytes_each, void* dst, void* sink, int width, int group,
                       int write, int64_t tile_bytes, void* stream) {
  if (!srcs || !sink || bytes_each < 16) return -1;
  SrcTable t;
  for (int k = 0; k < 128; ++k) t.p[k] = srcs[k];
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n = bytes_each / width;
  const int64_t tv = tile_bytes > 0 ? tile_bytes / width : 0, sv = tv * 128;
  const dim3 g(static_cast<unsigned>((n + 63) / 64)), b(64);
  uint32_t* sk = static_cast<uint32_t*>(sink);
#define DLP_MU(V, G)                                                                                          \
  do {                                                                                                        \
    if (write)                                                                                                \
      hipLaunchKernelGGL((mread_unrolled_kernel<V, G, true>), g, b, 0, s, t, n, static_cast<V*>(dst), sk, tv, sv); \
    else                                                                                                      \
      hipLaunchKernelGGL((mread_unrolled_kernel<V, G, false>), g, b, 0, s, t, n, static_cast<V*>(dst), sk, tv, sv); \
  } while (0)
  if (width == 8 && group == 16) DLP_MU(u32x2, 16);
  else if (width == 8 && group == 32) DLP_MU(u32x2, 32);
  else if (width == 16 && group == 16) DLP_MU(u32x4, 16);
  else if (width == 4 && group == 64) DLP_MU(uint32_t, 64);
  else return -1;
#undef DLP_MU
  return static_cast<int>(hipGetLastError());
}

// The LDS-DMA north-star probe (ldsdma_tiled8_kernel): slab = [tiles][8][4096] f32, w8 = 8
// fp32 weights, n_elems per peer (units of 256 computed; the tail is not), stages in {2, 3, 4, 6},
// grid = persistent one-wave workgroups (<= 0: 256 CUs x the stage's LDS-limited occupancy).
int dlp_ldsdma_tiled8(const void* slab, const float* w8, int64_t n_elems, void* out, int stages, int grid,
                      void* stream) {
  if (!slab || !w8 || !out || n_elems < 256) return -1;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n_units = n_elems / 256;
  const float* sl = static_cast<const float*>(slab);
  float* o = static_cast<float*>(out);
#define DLP_LD(SV)                                                                                               \
  do {                                                                                                           \
    const int g = grid > 0 ? grid : 256 * (160 / (8 * (SV)));                                                    \
    hipLaunchKernelGGL((ldsdma_tiled8_kernel<SV>), dim3(g), dim3(64), 0, s, sl, w8[0], w8[1], w8[2], w8[3], w8[4], \
                       w8[5], w8[6], w8[7], n_units, o);                                                         \
  } while (0)
  switch (stages) {
    case 2: DLP_LD(2); break;
    case 3: DLP_LD(3); break;
    case 4: DLP_LD(4); break;
    case 6: DLP_LD(6); break;
    default: return -1;
  }
#undef DLP_LD
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
