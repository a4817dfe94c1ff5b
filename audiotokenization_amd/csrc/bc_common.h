// Shared device helpers for the BigCodec gfx950 kernels.
//
// Every kernel in this library computes in fp32.  The whole library is compiled with
// -ffp-contract=off so that elementwise expressions round exactly where the reference's torch
// expressions round (an explicit fmaf() is used wherever a fused multiply-add is intended).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));

#define BC_OK 0
#define BC_ERR_ARG 1
#define BC_ERR_LAUNCH 2
#define BC_ERR_UNSUPPORTED 3

#define BC_CHECK_LAUNCH()                                   \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return BC_ERR_LAUNCH;             \
  } while (0)

namespace bc {

// SnakeBeta (vq/activations.py:107-118):  x + (1/(exp(b)+1e-9)) * sin(x*exp(a))^2.
// alpha_exp = exp(a) and inv_beta = 1/(exp(b)+1e-9) are precomputed per channel on the host with
// the same torch CPU expressions the reference evaluates, so only the per-element part runs here:
// t = x*alpha; s = sin(t); y = x + inv_beta*(s*s)   (pow(s,2) == s*s in torch).
__device__ __forceinline__ float snake(float x, float alpha_exp, float inv_beta) {
  float s = sinf(x * alpha_exp);
  return x + inv_beta * (s * s);
}

// Bijective XCD-aware remap of a 1-D workgroup id (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): workgroups that the dispatcher deals to the same XCD (ids b, b+8, b+16, ...) receive
// consecutive logical ids, so neighbouring tiles that share an input panel share one L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8, loc = orig / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

__device__ __forceinline__ float sigmoidf_ref(float x) { return 1.0f / (1.0f + expf(-x)); }

// splitmix64 finalizer (SURVEY.md §8(d) synthetic input spec).
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace bc
