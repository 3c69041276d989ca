// primitive check: xor_tree / add_xor_swap (enf_train.h) against the __shfl_xor butterfly, float and double
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "enf_train.h"
using namespace enf;
template <typename T>
__global__ void k(const T* in, T* out, int P) {
  const int l = threadIdx.x;
  T v = in[l], w = in[l];
  for (int m = P / 2; m >= 1; m >>= 1) w += __shfl_xor(w, m);
  out[l] = xor_tree(v, P);
  out[64 + l] = w;
  out[128 + l] = add_xor_swap<16>(in[l]);
  out[192 + l] = in[l] + __shfl_xor(in[l], 16);
  out[256 + l] = add_xor_swap<32>(in[l]);
  out[320 + l] = in[l] + __shfl_xor(in[l], 32);
}
template <typename T>
int run(const char* name) {
  T h[64], o[384];
  for (int i = 0; i < 64; ++i) h[i] = (T)((rand() % 100000) / 997.0 - 50.0);
  T *din, *dout;
  hipMalloc(&din, sizeof h); hipMalloc(&dout, sizeof o);
  hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  int bad = 0;
  for (int P = 1; P <= 64; P <<= 1) {
    hipLaunchKernelGGL(k<T>, dim3(1), dim3(64), 0, 0, din, dout, P);
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    int b1 = memcmp(o, o + 64, 64 * sizeof(T)) != 0, b2 = memcmp(o + 128, o + 192, 64 * sizeof(T)) != 0,
        b3 = memcmp(o + 256, o + 320, 64 * sizeof(T)) != 0;
    printf("%s P=%2d xor_tree %s swap16 %s swap32 %s  (lane0 %g vs %g, lane5 %g vs %g)\n", name, P, b1 ? "DIFF" : "ok",
           b2 ? "DIFF" : "ok", b3 ? "DIFF" : "ok", (double)o[0], (double)o[64], (double)o[5], (double)o[69]);
    bad |= b1 | b2 | b3;
  }
  return bad;
}
int main() { return run<float>("f32") | run<double>("f64"); }
