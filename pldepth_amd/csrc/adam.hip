// Fused Adam(amsgrad=True) over one flat fp32 parameter buffer.
//
// Replaces keras.optimizers.Adam(learning_rate, amsgrad=True) (pldepth/PLDepth.py:133), which TF
// applies per variable as ResourceApplyAdamWithAmsgrad (one launch per trainable tensor, ~120 for
// ff_effnet). Same update form as the TF functor:
//   alpha = lr*sqrt(1-b2^t)/(1-b1^t)   (host, fp32 like Keras' _prepare_local)
//   m += (g-m)*(1-b1); v += (g*g-v)*(1-b2); vhat = max(vhat, v); p -= m*alpha/(sqrt(vhat)+eps)
// HBM-bound: 5 reads + 4 writes of 4 B per parameter.
#include <cmath>

#include "common.h"

namespace pld {

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, float& vh,
                                         float alpha, float omb1, float omb2, float eps) {
  m += (g - m) * omb1;
  v += (g * g - v) * omb2;
  vh = fmaxf(vh, v);
  p -= (m * alpha) / (sqrtf(vh) + eps);
}

__global__ __launch_bounds__(256) void adam_amsgrad_kernel(float* __restrict__ p,
                                                           const float* __restrict__ g,
                                                           float* __restrict__ m,
                                                           float* __restrict__ v,
                                                           float* __restrict__ vh, long n4,
                                                           long n, float alpha, float omb1,
                                                           float omb2, float eps, float gs) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 P = reinterpret_cast<float4*>(p)[i];
    float4 G = reinterpret_cast<const float4*>(g)[i];
    float4 M = reinterpret_cast<float4*>(m)[i];
    float4 V = reinterpret_cast<float4*>(v)[i];
    float4 H = reinterpret_cast<float4*>(vh)[i];
    adam_one(P.x, G.x * gs, M.x, V.x, H.x, alpha, omb1, omb2, eps);
    adam_one(P.y, G.y * gs, M.y, V.y, H.y, alpha, omb1, omb2, eps);
    adam_one(P.z, G.z * gs, M.z, V.z, H.z, alpha, omb1, omb2, eps);
    adam_one(P.w, G.w * gs, M.w, V.w, H.w, alpha, omb1, omb2, eps);
    reinterpret_cast<float4*>(p)[i] = P;
    reinterpret_cast<float4*>(m)[i] = M;
    reinterpret_cast<float4*>(v)[i] = V;
    reinterpret_cast<float4*>(vh)[i] = H;
  }
  // scalar tail (n not a multiple of 4)
  const long t = n4 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) adam_one(p[t], g[t] * gs, m[t], v[t], vh[t], alpha, omb1, omb2, eps);
}

__global__ __launch_bounds__(256) void adam_amsgrad_dev_kernel(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
    float* __restrict__ v, float* __restrict__ vh, long n4, long n, const float* __restrict__ lr,
    const int64_t* __restrict__ step, float beta1, float beta2, float eps, float gs) {
  const float t = (float)step[0];
  const float alpha = lr[0] * sqrtf(1.0f - powf(beta2, t)) / (1.0f - powf(beta1, t));
  const float omb1 = 1.0f - beta1, omb2 = 1.0f - beta2;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 P = reinterpret_cast<float4*>(p)[i];
    float4 G = reinterpret_cast<const float4*>(g)[i];
    float4 M = reinterpret_cast<float4*>(m)[i];
    float4 V = reinterpret_cast<float4*>(v)[i];
    float4 H = reinterpret_cast<float4*>(vh)[i];
    adam_one(P.x, G.x * gs, M.x, V.x, H.x, alpha, omb1, omb2, eps);
    adam_one(P.y, G.y * gs, M.y, V.y, H.y, alpha, omb1, omb2, eps);
    adam_one(P.z, G.z * gs, M.z, V.z, H.z, alpha, omb1, omb2, eps);
    adam_one(P.w, G.w * gs, M.w, V.w, H.w, alpha, omb1, omb2, eps);
    reinterpret_cast<float4*>(p)[i] = P;
    reinterpret_cast<float4*>(m)[i] = M;
    reinterpret_cast<float4*>(v)[i] = V;
    reinterpret_cast<float4*>(vh)[i] = H;
  }
  const long t4 = n4 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t4 < n) adam_one(p[t4], g[t4] * gs, m[t4], v[t4], vh[t4], alpha, omb1, omb2, eps);
}

__global__ void step_increment_kernel(int64_t* s) { s[0] += 1; }
__global__ void set_scalar_kernel(float* d, float v) { d[0] = v; }

}  // namespace pld

extern "C" int pld_adam_amsgrad_dev(float* param, const float* grad, float* m, float* v,
                                    float* vhat, int64_t n, const float* lr_dev,
                                    const int64_t* step_dev, float beta1, float beta2, float eps,
                                    float grad_scale, void* stream) {
  using namespace pld;
  PLD_CHECK_ARG(param && grad && m && v && vhat && lr_dev && step_dev,
                "pld_adam_amsgrad_dev: null pointer");
  PLD_CHECK_ARG(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v |
                 (uintptr_t)vhat) % 16 == 0,
                "pld_adam_amsgrad_dev: buffers must be 16-byte aligned");
  if (n <= 0) return PLD_OK;
  const long n4 = n / 4;
  const unsigned grid = (unsigned)std::min<long>(std::max<long>(cdiv(n4, 256), 1), 4096);
  adam_amsgrad_dev_kernel<<<grid, 256, 0, as_stream(stream)>>>(
      param, grad, m, v, vhat, n4, n, lr_dev, step_dev, beta1, beta2, eps, grad_scale);
  return check_launch("adam_amsgrad_dev_kernel");
}

extern "C" int pld_step_increment(int64_t* step_dev, void* stream) {
  using namespace pld;
  PLD_CHECK_ARG(step_dev, "pld_step_increment: null pointer");
  step_increment_kernel<<<1, 1, 0, as_stream(stream)>>>(step_dev);
  return check_launch("step_increment_kernel");
}

extern "C" int pld_set_scalar_f32(float* dev, float value, void* stream) {
  using namespace pld;
  PLD_CHECK_ARG(dev, "pld_set_scalar_f32: null pointer");
  set_scalar_kernel<<<1, 1, 0, as_stream(stream)>>>(dev, value);
  return check_launch("set_scalar_kernel");
}

extern "C" int pld_adam_amsgrad(float* param, const float* grad, float* m, float* v, float* vhat,
                                int64_t n, float lr, float beta1, float beta2, float eps,
                                int64_t step, float grad_scale, void* stream) {
  using namespace pld;
  PLD_CHECK_ARG(param && grad && m && v && vhat, "pld_adam_amsgrad: null pointer");
  PLD_CHECK_ARG(n >= 0 && step >= 1, "pld_adam_amsgrad: bad n=%lld step=%lld", (long long)n,
                (long long)step);
  PLD_CHECK_ARG(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v |
                 (uintptr_t)vhat) % 16 == 0,
                "pld_adam_amsgrad: buffers must be 16-byte aligned");
  if (n == 0) return PLD_OK;
  // Keras: local_step = iterations + 1; beta powers and alpha in the variable dtype (float32)
  const float b1p = powf(beta1, (float)step);
  const float b2p = powf(beta2, (float)step);
  const float alpha = lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
  const long n4 = n / 4;
  const unsigned grid = (unsigned)std::min<long>(std::max<long>(cdiv(n4, 256), 1), 4096);
  adam_amsgrad_kernel<<<grid, 256, 0, as_stream(stream)>>>(param, grad, m, v, vhat, n4, n, alpha,
                                                           1.0f - beta1, 1.0f - beta2, eps,
                                                           grad_scale);
  return check_launch("adam_amsgrad_kernel");
}
