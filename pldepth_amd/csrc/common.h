// Shared helpers for the PLDepth HIP/CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/pldepth_hip.h"

namespace pld {

// ---- error plumbing (C-ABI entry points return an int status; text via pld_last_error) ----
void set_error(const char* fmt, ...);
int check_launch(const char* what);

#define PLD_CHECK_ARG(cond, ...)                                                          \
  do {                                                                                   \
    if (!(cond)) {                                                                       \
      ::pld::set_error(__VA_ARGS__);                                                     \
      return PLD_ERR_ARG;                                                                \
    }                                                                                    \
  } while (0)

#define PLD_HIP(call)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess) {                                                              \
      ::pld::set_error("%s failed: %s", #call, hipGetErrorString(e_));                    \
      return PLD_ERR_HIP;                                                                \
    }                                                                                    \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }
inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// ---- fp32 operations rounded on their own ----
// HIP's __fmul_rn / __fadd_rn are the plain operators (clang's HIP math header), which hipcc's
// default -ffp-contract=fast-honor-pragmas may fuse into one fma with a neighbouring add. These
// never fuse: for arithmetic that must round like the reference's separate NumPy / Keras ops
// (a drop-connect product then the residual sum; np.linspace's arange * step + start).
__device__ __forceinline__ float mul_rn(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float add_rn(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}

// ---- activations (Keras semantics) ----
enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_SWISH = 2, ACT_SIGMOID = 3 };

// v_exp_f32 + v_rcp_f32 (1 ulp each): the IEEE division's scale/fixup sequence cost ~10
// instructions per activation in the kernels that re-apply BN + activation on every read
__device__ __forceinline__ float sigmoidf_(float z) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-z));
}

__device__ __forceinline__ float act_fwd(int act, float z) {
  switch (act) {
    case ACT_RELU: return z > 0.f ? z : 0.f;
    case ACT_SWISH: return z * sigmoidf_(z);
    case ACT_SIGMOID: return sigmoidf_(z);
    default: return z;
  }
}

// derivative of act at pre-activation z
__device__ __forceinline__ float act_grad(int act, float z) {
  switch (act) {
    case ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case ACT_SWISH: {
      float s = sigmoidf_(z);
      return s * (1.f + z * (1.f - s));
    }
    case ACT_SIGMOID: {
      float s = sigmoidf_(z);
      return s * (1.f - s);
    }
    default: return 1.f;
  }
}

// ---- fast unsigned division by a runtime-constant divisor (host-built magic numbers) ----
struct FastDiv {
  uint32_t d, m, s;
  FastDiv() : d(1), m(0), s(0) {}
  explicit FastDiv(uint32_t div) : d(div) {
    // q = (mulhi(n, m) + n) >> s, exact for 0 <= n < 2^31 (Granlund–Montgomery round-up magic)
    s = 0;
    while (s < 32 && (1u << s) < d) ++s;
    uint64_t one = 1;
    m = (uint32_t)(((one << 32) * ((one << s) - d)) / d + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    uint32_t t = __umulhi(n, m);
    return (t + n) >> s;
  }
  __device__ __forceinline__ uint32_t mod(uint32_t n, uint32_t q) const { return n - q * d; }
};

// 16-byte streaming store (nt): for outputs written once and read by a later kernel. Measured on
// the BN apply (401408 x 144, back-to-back launches): 83.6 -> 66.9 us, 5.5 -> 6.9 TB/s
// (profiles/r04_store_policy_ab.txt; write-through sc1 stores: no gain)
__device__ __forceinline__ void st_nt4(float* p, float4 v) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const f32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<f32x4*>(p));
}

// wave-level reductions (wave64)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace pld
