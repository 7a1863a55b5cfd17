/* c_abi_demo.c — the C ABI of libdlagg.so used from plain C (no Python, no torch).
 *
 * Builds with gcc against the HIP runtime for device allocation only:
 *   gcc -std=c11 -O2 -ffp-contract=off tests/c_abi_demo.c -Iinclude -I/opt/rocm/include \
 *       -D__HIP_PLATFORM_AMD__ -Ldecentralized-learning_amd/lib -ldlagg -L/opt/rocm/lib -lamdhip64 -o c_abi_demo
 * Runs FedAvg (dla_wsum, a dla_plan with changed weights, the bucket-sharded dla_wsum_sharded and
 * the tile-interleaved dla_wsum_slab_tiled, host-resident peers through dla_host_round_* and the
 * chunked dla_host_reduce, peers staged by dla_slab_stage, peers of several dtypes through
 * dla_wsum_mixed) and the
 * teacher-logit mean (dla_mean) on N peers and checks every element bit-for-bit against the reference's
 * sequential arithmetic written out in C (fedavg.py:21-25).  Exit status 0 = all equal.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dlagg.h"

#define CHECK_HIP(x)                                                      \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));      \
      return 2;                                                           \
    }                                                                     \
  } while (0)

#define CHECK_DLA(x)                                                      \
  do {                                                                    \
    int r_ = (x);                                                         \
    if (r_ != DLA_OK) {                                                   \
      fprintf(stderr, "%s failed (%d): %s\n", #x, r_, dla_last_error());  \
      return 3;                                                           \
    }                                                                     \
  } while (0)

/* RNE float -> bf16 bits (NaN -> 0x7FC0), and back */
static uint16_t to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if (isnan(f)) return 0x7FC0;
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

static float from_bf16(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static int same_f32(float a, float b) {
  uint32_t x, y;
  memcpy(&x, &a, 4);
  memcpy(&y, &b, 4);
  return (isnan(a) && isnan(b)) || x == y;
}

int main(void) {
  enum { N = 5 };
  const int64_t P = 1000003; /* ragged: not a multiple of the 16-byte chunk */
  double w[N] = {0.1, 0.25, 0.3, 0.2, 0.15};
  float* host[N];
  void* dev[N];
  float* out_host = (float*)malloc(sizeof(float) * P);
  void* dev_out;
  unsigned s = 12345u;
  if (dla_version() != DLA_ABI_VERSION) {
    fprintf(stderr, "ABI version mismatch\n");
    return 4;
  }
  for (int k = 0; k < N; ++k) {
    host[k] = (float*)malloc(sizeof(float) * P);
    for (int64_t j = 0; j < P; ++j) {
      s = s * 1664525u + 1013904223u;
      host[k][j] = ((float)(s >> 8) / 16777216.0f - 0.5f) * 0.1f;
    }
    CHECK_HIP(hipMalloc(&dev[k], sizeof(float) * P));
    CHECK_HIP(hipMemcpy(dev[k], host[k], sizeof(float) * P, hipMemcpyHostToDevice));
  }
  CHECK_HIP(hipMalloc(&dev_out, sizeof(float) * P));

  /* 1. dla_wsum on the default stream */
  CHECK_DLA(dla_wsum(DLA_F32, (const void* const*)dev, w, N, P, dev_out, NULL));
  CHECK_HIP(hipMemcpy(out_host, dev_out, sizeof(float) * P, hipMemcpyDeviceToHost));
  for (int64_t j = 0; j < P; ++j) {
    volatile float acc = host[0][j] * 0.0f;
    for (int k = 0; k < N; ++k) {
      volatile float prod = (float)w[k] * host[k][j];
      acc = acc + prod;
    }
    if (!same_f32(acc, out_host[j])) {
      fprintf(stderr, "dla_wsum mismatch at %lld\n", (long long)j);
      return 1;
    }
  }

  /* 2. a prepared plan, relaunched with new weights */
  dla_plan_t* plan = NULL;
  CHECK_DLA(dla_plan_create(&plan, DLA_F32, (const void* const*)dev, w, N, P, dev_out, NULL));
  double w2[N] = {1.0, -0.5, 0.0, 2.0, 0.125};
  CHECK_DLA(dla_plan_set_weights(plan, w2));
  CHECK_DLA(dla_plan_launch(plan, NULL));
  CHECK_HIP(hipMemcpy(out_host, dev_out, sizeof(float) * P, hipMemcpyDeviceToHost));
  dla_plan_destroy(plan);
  for (int64_t j = 0; j < P; ++j) {
    volatile float acc = host[0][j] * 0.0f;
    for (int k = 0; k < N; ++k) {
      volatile float prod = (float)w2[k] * host[k][j];
      acc = acc + prod;
    }
    if (!same_f32(acc, out_host[j])) {
      fprintf(stderr, "dla_plan mismatch at %lld\n", (long long)j);
      return 1;
    }
  }

  /* 3. teacher-logit mean */
  CHECK_DLA(dla_mean(DLA_F32, (const void* const*)dev, N, P, dev_out, NULL));
  CHECK_HIP(hipMemcpy(out_host, dev_out, sizeof(float) * P, hipMemcpyDeviceToHost));
  for (int64_t j = 0; j < P; ++j) {
    volatile float acc = 0.0f;
    for (int k = 0; k < N; ++k) acc = acc + host[k][j];
    volatile float mean = acc / (float)N;
    if (!same_f32(mean, out_host[j])) {
      fprintf(stderr, "dla_mean mismatch at %lld\n", (long long)j);
      return 1;
    }
  }

  /* 4. bucket-sharded over the GPUs of this process (dla_wsum_sharded): three shards, every
   *    one on device 0 here (ids may repeat), each writing its bucket straight into dev_out */
  {
    int ids[3] = {0, 0, 0};
    void* outs[3] = {dev_out, dev_out, dev_out};
    void* streams[3] = {NULL, NULL, NULL};
    CHECK_HIP(hipMemset(dev_out, 0xff, sizeof(float) * P));
    CHECK_DLA(dla_wsum_sharded(DLA_F32, 3, ids, (const void* const*)dev, w, N, P, outs, 0, streams));
    CHECK_HIP(hipMemcpy(out_host, dev_out, sizeof(float) * P, hipMemcpyDeviceToHost));
    for (int64_t j = 0; j < P; ++j) {
      volatile float acc = host[0][j] * 0.0f;
      for (int k = 0; k < N; ++k) {
        volatile float prod = (float)w[k] * host[k][j];
        acc = acc + prod;
      }
      if (!same_f32(acc, out_host[j])) {
        fprintf(stderr, "dla_wsum_sharded mismatch at %lld\n", (long long)j);
        return 1;
      }
    }
    CHECK_DLA(dla_shutdown());
  }

  /* 5. the tile-interleaved slab (dla_wsum_slab_tiled): row k's tile t at (t * N + k) * T */
  {
    const int64_t T = dla_slab_tile_elems(DLA_F32, N, P);
    const int64_t n_t = (P + T - 1) / T;
    float* tiled = (float*)calloc((size_t)(n_t * N * T), sizeof(float));
    void* dev_tiled;
    for (int k = 0; k < N; ++k)
      for (int64_t j = 0; j < P; ++j) tiled[((j / T) * N + k) * T + j % T] = host[k][j];
    CHECK_HIP(hipMalloc(&dev_tiled, sizeof(float) * (size_t)(n_t * N * T)));
    CHECK_HIP(hipMemcpy(dev_tiled, tiled, sizeof(float) * (size_t)(n_t * N * T), hipMemcpyHostToDevice));
    CHECK_DLA(dla_wsum_slab_tiled(DLA_F32, dev_tiled, T, N, w, N, P, dev_out, NULL, NULL));
    CHECK_HIP(hipMemcpy(out_host, dev_out, sizeof(float) * P, hipMemcpyDeviceToHost));
    for (int64_t j = 0; j < P; ++j) {
      volatile float acc = host[0][j] * 0.0f;
      for (int k = 0; k < N; ++k) {
        volatile float prod = (float)w[k] * host[k][j];
        acc = acc + prod;
      }
      if (!same_f32(acc, out_host[j])) {
        fprintf(stderr, "dla_wsum_slab_tiled mismatch at %lld\n", (long long)j);
        return 1;
      }
    }
    CHECK_HIP(hipFree(dev_tiled));
    free(tiled);
  }

  /* 6. peers in host memory (dla_host_round_start / _finish): each peer as two tensors, packed
   *    into page-locked rows the kernel reads across PCIe, unpacked into two host outputs */
  {
    const int64_t split = 4099, numels[2] = {split, P - split};
    const int64_t pitch = (P + 63) / 64 * 64;
    const void* tensors[2 * N];
    void *rows, *result;
    float* outs_host[2] = {out_host, out_host + split};
    for (int k = 0; k < N; ++k) {
      tensors[2 * k] = host[k];
      tensors[2 * k + 1] = host[k] + split;
    }
    CHECK_HIP(hipHostMalloc(&rows, sizeof(float) * (size_t)(N * pitch), hipHostMallocDefault));
    CHECK_HIP(hipHostMalloc(&result, sizeof(float) * (size_t)pitch, hipHostMallocDefault));
    memset(out_host, 0xff, sizeof(float) * P);
    CHECK_DLA(dla_host_round_start(DLA_F32, N, 2, tensors, numels, w, rows, pitch, result, NULL));
    CHECK_DLA(dla_host_round_finish(DLA_F32, 2, numels, result, (void* const*)outs_host, NULL));
    for (int64_t j = 0; j < P; ++j) {
      volatile float acc = host[0][j] * 0.0f;
      for (int k = 0; k < N; ++k) {
        volatile float prod = (float)w[k] * host[k][j];
        acc = acc + prod;
      }
      if (!same_f32(acc, out_host[j])) {
        fprintf(stderr, "dla_host_round mismatch at %lld\n", (long long)j);
        return 1;
      }
    }
    /* pageable rows are refused before any launch */
    if (dla_host_round_start(DLA_F32, N, 2, tensors, numels, w, out_host, pitch, result, NULL) != DLA_E_INVALID) {
      fprintf(stderr, "expected DLA_E_INVALID for pageable rows\n");
      return 1;
    }
    CHECK_HIP(hipHostFree(rows));
    CHECK_HIP(hipHostFree(result));
  }

  /* 7. a large round of host peers streamed in chunks (dla_host_reduce): the same two tensors per
   *    peer, 8 192-element chunks (the last one partial), two streams */
  {
    const int64_t split = 4099, numels[2] = {split, P - split}, chunk = 8192;
    const void* tensors[2 * N];
    void *h_stage, *d_stage, *h_out, *d_out2;
    void* outs_host[2] = {out_host, out_host + split};
    hipStream_t st, cst;
    for (int k = 0; k < N; ++k) {
      tensors[2 * k] = host[k];
      tensors[2 * k + 1] = host[k] + split;
    }
    CHECK_HIP(hipStreamCreate(&st));
    CHECK_HIP(hipStreamCreate(&cst));
    CHECK_HIP(hipHostMalloc(&h_stage, sizeof(float) * (size_t)(2 * N * chunk), hipHostMallocDefault));
    CHECK_HIP(hipHostMalloc(&h_out, sizeof(float) * (size_t)(2 * chunk), hipHostMallocDefault));
    CHECK_HIP(hipMalloc(&d_stage, sizeof(float) * (size_t)(2 * N * chunk)));
    CHECK_HIP(hipMalloc(&d_out2, sizeof(float) * (size_t)(2 * chunk)));
    memset(out_host, 0xff, sizeof(float) * P);
    /* in two calls over [0, 300 007) and [300 007, P): the buckets of a round sharded over two GPUs */
    CHECK_DLA(dla_host_reduce(DLA_F32, N, 2, tensors, numels, w, outs_host, 0, 300007, chunk, h_stage, d_stage,
                              h_out, d_out2, st, cst));
    CHECK_DLA(dla_host_reduce(DLA_F32, N, 2, tensors, numels, w, outs_host, 300007, P, chunk, h_stage, d_stage,
                              h_out, d_out2, st, cst));
    for (int64_t j = 0; j < P; ++j) {
      volatile float acc = host[0][j] * 0.0f;
      for (int k = 0; k < N; ++k) {
        volatile float prod = (float)w[k] * host[k][j];
        acc = acc + prod;
      }
      if (!same_f32(acc, out_host[j])) {
        fprintf(stderr, "dla_host_reduce mismatch at %lld\n", (long long)j);
        return 1;
      }
    }
    /* the same round launched on a library thread, its outputs published after the launch (ABI v9) */
    {
      void* late_outs[2] = {NULL, NULL};
      int ready = 0;
      dla_host_job_t* job = NULL;
      memset(out_host, 0xff, sizeof(float) * P);
      CHECK_DLA(dla_host_reduce_launch(0, DLA_F32, N, 2, tensors, numels, w, late_outs, &ready, 0, P, chunk, h_stage,
                                       d_stage, h_out, d_out2, st, cst, &job));
      late_outs[0] = out_host;
      late_outs[1] = out_host + split;
      __atomic_store_n(&ready, 1, __ATOMIC_RELEASE);
      CHECK_DLA(dla_host_reduce_join(job));
      for (int64_t j = 0; j < P; ++j) {
        volatile float acc = host[0][j] * 0.0f;
        for (int k = 0; k < N; ++k) {
          volatile float prod = (float)w[k] * host[k][j];
          acc = acc + prod;
        }
        if (!same_f32(acc, out_host[j])) {
          fprintf(stderr, "dla_host_reduce_launch mismatch at %lld\n", (long long)j);
          return 1;
        }
      }
      /* abandoned: the job drains and reports it */
      ready = 0;
      CHECK_DLA(dla_host_reduce_launch(0, DLA_F32, N, 2, tensors, numels, w, late_outs, &ready, 0, P, chunk, h_stage,
                                       d_stage, h_out, d_out2, st, cst, &job));
      __atomic_store_n(&ready, -1, __ATOMIC_RELEASE);
      if (dla_host_reduce_join(job) != DLA_E_INVALID || !strstr(dla_last_error(), "abandoned")) {
        fprintf(stderr, "expected an abandoned job to fail with DLA_E_INVALID\n");
        return 1;
      }
    }
    /* a pageable staging buffer is refused before any copy */
    if (dla_host_reduce(DLA_F32, N, 2, tensors, numels, w, outs_host, 0, P, chunk, out_host, d_stage, h_out, d_out2,
                        st, cst) != DLA_E_INVALID) {
      fprintf(stderr, "expected DLA_E_INVALID for a pageable h_stage\n");
      return 1;
    }
    CHECK_HIP(hipHostFree(h_stage));
    CHECK_HIP(hipHostFree(h_out));
    CHECK_HIP(hipFree(d_stage));
    CHECK_HIP(hipFree(d_out2));
    CHECK_HIP(hipStreamDestroy(st));
    CHECK_HIP(hipStreamDestroy(cst));
  }

  /* 8. peers staged into a tile-interleaved slab row by row (dla_slab_stage: host -> device, one 2D
   *    copy per row for the whole tiles) and reduced from it; a range past the slab is refused */
  {
    const int64_t T = dla_slab_tile_elems(DLA_F32, N, P);
    const int64_t n_t = (P + T - 1) / T;
    void* dev_tiled;
    CHECK_HIP(hipMalloc(&dev_tiled, sizeof(float) * (size_t)(n_t * N * T)));
    for (int k = 0; k < N; ++k)
      CHECK_DLA(dla_slab_stage(DLA_F32, dev_tiled, T, N, n_t, k, 0, host[k], P, NULL));
    CHECK_HIP(hipDeviceSynchronize());
    CHECK_DLA(dla_wsum_slab_tiled(DLA_F32, dev_tiled, T, N, w, N, P, dev_out, NULL, NULL));
    CHECK_HIP(hipMemcpy(out_host, dev_out, sizeof(float) * P, hipMemcpyDeviceToHost));
    for (int64_t j = 0; j < P; ++j) {
      volatile float acc = host[0][j] * 0.0f;
      for (int k = 0; k < N; ++k) {
        volatile float prod = (float)w[k] * host[k][j];
        acc = acc + prod;
      }
      if (!same_f32(acc, out_host[j])) {
        fprintf(stderr, "dla_slab_stage + dla_wsum_slab_tiled mismatch at %lld\n", (long long)j);
        return 1;
      }
    }
    if (dla_slab_stage(DLA_F32, dev_tiled, T, N, n_t, 0, n_t * T - 10, host[0], 11, NULL) != DLA_E_INVALID) {
      fprintf(stderr, "expected DLA_E_INVALID for a range past the slab\n");
      return 1;
    }
    CHECK_HIP(hipFree(dev_tiled));
  }

  /* 9. peers of several dtypes (dla_wsum_mixed): models[0] f32, then a peer in f64 and one in bf16 —
   *    fedavg.py:25 rounds w * p in the peer's dtype and adds in the promoted type (f64 with the f64
   *    peer, f32 with the bf16 one), rounding the sum to f32 */
  {
    double* h64 = (double*)malloc(sizeof(double) * P);
    uint16_t* h16 = (uint16_t*)malloc(sizeof(uint16_t) * P);
    void *d64, *d16;
    for (int64_t j = 0; j < P; ++j) {
      h64[j] = (double)host[1][j] * 1.0000001;
      h16[j] = to_bf16(host[2][j]);
    }
    CHECK_HIP(hipMalloc(&d64, sizeof(double) * P));
    CHECK_HIP(hipMalloc(&d16, sizeof(uint16_t) * P));
    CHECK_HIP(hipMemcpy(d64, h64, sizeof(double) * P, hipMemcpyHostToDevice));
    CHECK_HIP(hipMemcpy(d16, h16, sizeof(uint16_t) * P, hipMemcpyHostToDevice));
    const void* mp[3] = {dev[0], d64, d16};
    const int dts[3] = {DLA_F32, DLA_F64, DLA_BF16};
    const double mw[3] = {0.2, 0.3, 0.5};
    CHECK_DLA(dla_wsum_mixed(DLA_F32, dts, mp, mw, 3, P, dev_out, NULL));
    CHECK_HIP(hipMemcpy(out_host, dev_out, sizeof(float) * P, hipMemcpyDeviceToHost));
    for (int64_t j = 0; j < P; ++j) {
      volatile float acc = host[0][j] * 0.0f;
      volatile float p0 = (float)mw[0] * host[0][j];
      acc = acc + p0;
      volatile double p1 = mw[1] * h64[j];
      volatile double s1 = (double)acc + p1;
      acc = (float)s1;
      volatile float p2f = (float)mw[2] * from_bf16(h16[j]);
      const float p2 = from_bf16(to_bf16(p2f));
      acc = acc + p2;
      if (!same_f32(acc, out_host[j])) {
        fprintf(stderr, "dla_wsum_mixed mismatch at %lld\n", (long long)j);
        return 1;
      }
    }
    const int bad[3] = {DLA_BF16, DLA_F64, DLA_BF16};  /* peers[0] must carry out_dtype */
    if (dla_wsum_mixed(DLA_F32, bad, mp, mw, 3, P, dev_out, NULL) != DLA_E_INVALID) {
      fprintf(stderr, "expected DLA_E_INVALID for peers[0] not in out_dtype\n");
      return 1;
    }
    CHECK_HIP(hipFree(d64));
    CHECK_HIP(hipFree(d16));
    free(h64);
    free(h16);
  }

  /* 10. errors come back as codes with a message */
  if (dla_wsum(DLA_F32, (const void* const*)dev, w, 0, P, dev_out, NULL) != DLA_E_INVALID ||
      strlen(dla_last_error()) == 0) {
    fprintf(stderr, "expected DLA_E_INVALID for n_peers = 0\n");
    return 1;
  }

  for (int k = 0; k < N; ++k) {
    CHECK_HIP(hipFree(dev[k]));
    free(host[k]);
  }
  CHECK_HIP(hipFree(dev_out));
  free(out_host);
  printf("c_abi_demo ok: dla_wsum, dla_plan, dla_mean, dla_wsum_sharded, dla_wsum_slab_tiled, dla_host_round, "
         "dla_host_reduce (+ launch / join), dla_slab_stage, dla_wsum_mixed "
         "bit-exact on %d peers "
         "x %lld fp32\n", N, (long long)P);
  return 0;
}
