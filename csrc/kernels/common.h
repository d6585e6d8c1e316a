// Common device helpers for the dtfe CDNA4 (gfx950) kernel library.
//
// Everything here is written for MI355X directly: 64-lane wavefronts, MFMA
// fragments, LDS address-space casts for the gfx950 transpose read.  No CUDA
// shims, no dual paths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>
#include <cstring>

namespace dtfe {

typedef uint16_t bf16;  // storage type for bfloat16

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ float bf2f(bf16 v) { return __uint_as_float(((uint32_t)v) << 16); }

// round-to-nearest-even fp32 -> bf16 on the gfx950 converter (v_cvt_pk_bf16_f32; NaN stays a quiet
// NaN).  The software rounding it replaces (bit test, add, select: ~5 VALU per value) was a third of
// the implicit-GEMM epilogue's vector instructions.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf16 f2bf(float f) { return __builtin_bit_cast(bf16, (__bf16)f); }

// two values, one instruction
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}

// Activation codes shared with the host side (ops/_lib.py mirrors these).
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2, ACT_TANH = 3 };

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ __forceinline__ float apply_act(float x, int act) {
  switch (act) {
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_SIGMOID: return sigmoidf_(x);
    case ACT_TANH: return tanhf(x);
    default: return x;
  }
}

// BatchNorm affine with ONE rounding, written out: y = x * scale + shift with scale = gamma * invstd,
// shift = beta - mean * scale.  Every kernel that forms a BN output or recomputes its ReLU mask from x
// (bn_apply, bn_finalize + the implicit-GEMM operand transform, the backward's mask from x, the stem's
// BN + pool) uses these, so the values agree bit for bit whatever the compiler would contract
__device__ __forceinline__ float bn_shift(float beta, float mean, float scale) { return __builtin_fmaf(-mean, scale, beta); }
__device__ __forceinline__ float bn_affine(float x, float scale, float shift) { return __builtin_fmaf(x, scale, shift); }

// derivative of the activation expressed through its OUTPUT y = act(z)
__device__ __forceinline__ float act_grad_from_out(float y, int act) {
  switch (act) {
    case ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case ACT_SIGMOID: return y * (1.f - y);
    case ACT_TANH: return 1.f - y * y;
    default: return 1.f;
  }
}

// 64-lane wave reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Counter-based hash RNG (deterministic, stateless): used for dropout masks,
// on-device batch sampling and synthetic data.  splitmix/murmur finaliser.
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t idx) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + idx * 0xD1B54A32D192ED03ull + 0x632BE59BD9B4E019ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)z;
}
__device__ __forceinline__ float hash_uniform(uint64_t seed, uint64_t idx) {
  return (hash_u32(seed, idx) >> 8) * (1.0f / 16777216.0f);  // [0,1)
}

// XCD-aware bijective remap of a flat workgroup id (cdna_hip_programming T1):
// consecutive logical tiles land on the same XCD so they share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nxcd = 8;
  if (nwg <= nxcd) return orig;
  int q = nwg / nxcd, r = nwg % nxcd;
  int xcd = orig % nxcd;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / nxcd;
}

// Ablation bits of one kernel family from DTFE_DIAG="key=bits[,key=bits...]" (keys: c1, c1w, ic,
// iw - the MNIST conv kernels' stage-skipping switches used by the bench/*_diag.py ablations)
inline int diag_bits(const char* key) {
  const char* e = std::getenv("DTFE_DIAG");
  const size_t n = std::strlen(key);
  while (e && *e) {
    if (!std::strncmp(e, key, n) && e[n] == '=') return std::atoi(e + n + 1);
    e = std::strchr(e, ',');
    if (e) ++e;
  }
  return 0;
}

}  // namespace dtfe
