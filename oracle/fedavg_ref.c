/*
 * fedavg_ref.c — plain-C restatement of the accdfl FedAvg reduce.  TEST INFRASTRUCTURE
 * ONLY: loaded by tests/ (as an independent second oracle, fast enough for the
 * full 8 x 25 M north-star size) and never by the product path.
 *
 * Follows /root/reference/accdfl/core/gradient_aggregation/fedavg.py:
 *   :14-17  weights already defaulted by the caller
 *   :21-22  acc = p0 * 0
 *   :23-25  for k in list order: acc = R(acc + R(W(w_k) * p_k))   (no FMA)
 * Build: gcc -O2 -ffp-contract=off -fno-fast-math -fopenmp -shared -fPIC
 * (oracle/Makefile).  Elements are independent, so the OpenMP split over elements
 * does not change any result; the peer order per element is the list order.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static inline float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

/* c10::BFloat16 round_to_nearest_even: NaN -> 0x7FC0, else RNE on the bits. */
static inline uint16_t f32_to_bf16(float f) {
  if (isnan(f)) return 0x7FC0;
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

void oracle_wsum_f32(const float* const* peers, const double* w, int n, int64_t len, float* out) {
  float wf[1024];
  const int nw = n < 1024 ? n : 1024;
  for (int k = 0; k < nw; ++k) wf[k] = (float)w[k];
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < len; ++j) {
    volatile float acc = peers[0][j] * 0.0f;
    for (int k = 0; k < n; ++k) {
      const float wk = k < 1024 ? wf[k] : (float)w[k];
      volatile float prod = wk * peers[k][j];
      acc = acc + prod;
    }
    out[j] = acc;
  }
}

void oracle_wsum_f64(const double* const* peers, const double* w, int n, int64_t len, double* out) {
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < len; ++j) {
    volatile double acc = peers[0][j] * 0.0;
    for (int k = 0; k < n; ++k) {
      volatile double prod = w[k] * peers[k][j];
      acc = acc + prod;
    }
    out[j] = acc;
  }
}

void oracle_wsum_bf16(const uint16_t* const* peers, const double* w, int n, int64_t len, uint16_t* out) {
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < len; ++j) {
    uint16_t acc = f32_to_bf16(bf16_to_f32(peers[0][j]) * 0.0f);
    for (int k = 0; k < n; ++k) {
      volatile float prod = (float)w[k] * bf16_to_f32(peers[k][j]);
      const uint16_t pb = f32_to_bf16(prod);
      volatile float sum = bf16_to_f32(acc) + bf16_to_f32(pb);
      acc = f32_to_bf16(sum);
    }
    out[j] = acc;
  }
}

/* f16 via _Float16 (gcc >= 12) is not available on gcc 11 / x86: restate the
 * IEEE binary16 conversions on the bits. */
static inline float f16_to_f32(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  const uint32_t exp = (h >> 10) & 0x1Fu;
  const uint32_t man = h & 0x3FFu;
  uint32_t u;
  if (exp == 0) {
    if (man == 0) {
      u = sign;
    } else { /* subnormal: value = man * 2^-24 */
      float f = ldexpf((float)man, -24);
      memcpy(&u, &f, 4);
      u |= sign;
    }
  } else if (exp == 31) {
    u = sign | 0x7F800000u | (man << 13);
  } else {
    u = sign | ((exp + 112u) << 23) | (man << 13);
  }
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static inline uint16_t f32_to_f16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  const uint16_t sign = (uint16_t)((u >> 16) & 0x8000u);
  const uint32_t a = u & 0x7FFFFFFFu;
  if (a > 0x7F800000u) return (uint16_t)(sign | 0x7E00u);     /* NaN */
  if (a >= 0x47800000u) {                                     /* >= 65536: overflow */
    /* values in [65520, 65536) round to inf as well; handled below by rounding */
    return (uint16_t)(sign | 0x7C00u);
  }
  if (a < 0x38800000u) { /* below the f16 normal range: subnormal or zero */
    /* value / 2^-24, rounded to nearest even integer */
    float af;
    memcpy(&af, &a, 4);
    const float scaled = af * 16777216.0f; /* exact: power of two */
    float r = nearbyintf(scaled);          /* default rounding mode: RNE */
    return (uint16_t)(sign | (uint16_t)r);
  }
  /* normal: keep 10 mantissa bits, RNE on the 13 dropped bits */
  uint32_t e = (a >> 23) - 112u;
  uint32_t m = a & 0x7FFFFFu;
  uint32_t h = (e << 10) | (m >> 13);
  const uint32_t rem = m & 0x1FFFu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h += 1u; /* may carry into exp / inf */
  return (uint16_t)(sign | h);
}

void oracle_wsum_f16(const uint16_t* const* peers, const double* w, int n, int64_t len, uint16_t* out) {
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < len; ++j) {
    uint16_t acc = f32_to_f16(f16_to_f32(peers[0][j]) * 0.0f);
    for (int k = 0; k < n; ++k) {
      volatile float prod = (float)w[k] * f16_to_f32(peers[k][j]);
      const uint16_t pb = f32_to_f16(prod);
      volatile float sum = f16_to_f32(acc) + f16_to_f32(pb);
      acc = f32_to_f16(sum);
    }
    out[j] = acc;
  }
}

/* Mixed dtypes (fedavg.py:25 when a peer's parameter has another dtype than models[0]'s): the
 * product rounded in the peer's dtype (op-math f32, f64 for an f64 peer), the sum in the promoted
 * type (f64 if either side is f64, else f32) rounded to the centre's dtype; an f64 sum reaches a
 * 16-bit centre through float, as torch's c10::BFloat16 / c10::Half(float) casts do.  Codes as
 * include/dlagg.h: 0 f32, 1 bf16, 2 f16, 3 f64.  The running value is kept as a double holding a
 * value of the centre's dtype exactly. */
static inline double mx_load(const void* p, int dt, int64_t j) {
  switch (dt) {
    case 0: return (double)((const float*)p)[j];
    case 1: return (double)bf16_to_f32(((const uint16_t*)p)[j]);
    case 2: return (double)f16_to_f32(((const uint16_t*)p)[j]);
    default: return ((const double*)p)[j];
  }
}

static inline float mx_round32(float f, int dt) {
  if (dt == 1) return bf16_to_f32(f32_to_bf16(f));
  if (dt == 2) return f16_to_f32(f32_to_f16(f));
  return f;
}

void oracle_wsum_mixed(int out_dt, const int* dts, const void* const* peers, const double* w, int n, int64_t len,
                       void* out) {
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < len; ++j) {
    volatile double acc;
    const double x0 = mx_load(peers[0], dts[0], j);
    if (out_dt == 3) {
      acc = x0 * 0.0;
    } else {
      volatile float z = (float)x0 * 0.0f;
      acc = z;
    }
    for (int k = 0; k < n; ++k) {
      const int dk = dts[k];
      const double x = mx_load(peers[k], dk, j);
      volatile double prod;
      if (dk == 3) {
        prod = w[k] * x;
      } else {
        volatile float p32 = (float)w[k] * (float)x;
        prod = mx_round32(p32, dk);
      }
      if (out_dt == 3 || dk == 3) {
        volatile double s = acc + prod;
        if (out_dt == 3) {
          acc = s;
        } else {
          volatile float s32 = (float)s;
          acc = mx_round32(s32, out_dt);
        }
      } else {
        volatile float s32 = (float)acc + (float)prod;
        acc = mx_round32(s32, out_dt);
      }
    }
    switch (out_dt) {
      case 0: ((float*)out)[j] = (float)acc; break;
      case 1: ((uint16_t*)out)[j] = f32_to_bf16((float)acc); break;
      case 2: ((uint16_t*)out)[j] = f32_to_f16((float)acc); break;
      default: ((double*)out)[j] = acc; break;
    }
  }
}
