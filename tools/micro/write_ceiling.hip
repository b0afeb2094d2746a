// Micro-benchmark: the record-stream ceiling of the C4 block kernel.  12,500 workgroups of 256 threads each write a
// contiguous 14,336-B slab (32 blocks × 448 B of fp32 records) with 16-B non-temporal stores — the block kernel's
// store pattern with nothing else — and, in a second variant, also gather 4 bytes per lane from a 376-MB buffer
// (the image taps' volume) before storing.  Average per launch over 200 back-to-back launches (two HIP events).
// Diagnostic only.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool GATHER>
__global__ __launch_bounds__(256) void slab_kernel(f32x4* __restrict__ out, const unsigned char* __restrict__ img,
                                                   long long img_bytes, int slab16) {
  f32x4 v = {1.0f, 2.0f, 3.0f, (float)threadIdx.x};
  if (GATHER) {
    // four scattered byte loads per lane (the bilinear taps), folded into the stored value
    const unsigned long long h = (blockIdx.x * 2654435761ull) ^ (threadIdx.x * 40503ull);
    float s = 0.0f;
#pragma unroll
    for (int t = 0; t < 4; ++t) s += (float)img[(h * (t + 1) * 97ull) % (unsigned long long)img_bytes];
    v.x += s;
  }
  f32x4* dst = out + (long long)blockIdx.x * slab16;
  for (int i = threadIdx.x; i < slab16; i += 256) __builtin_nontemporal_store(v, dst + i);
}

int main() {
  const int wgs = 12500, slab = 14336, slab16 = slab / 16;
  const size_t out_bytes = (size_t)wgs * slab;
  const long long img_bytes = 376LL << 20;
  f32x4* out = nullptr;
  unsigned char* img = nullptr;
  if (hipMalloc(&out, out_bytes) != hipSuccess || hipMalloc(&img, img_bytes) != hipSuccess) return 1;
  (void)hipMemset(img, 7, img_bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int variant = 0; variant < 2; ++variant) {
    auto launch = [&] {
      if (variant == 0) slab_kernel<false><<<wgs, 256>>>(out, img, img_bytes, slab16);
      else slab_kernel<true><<<wgs, 256>>>(out, img, img_bytes, slab16);
    };
    for (int i = 0; i < 400; ++i) launch();  // clocks up
    (void)hipEventRecord(e0);
    const int n = 200;
    for (int i = 0; i < n; ++i) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double us = 1e3 * ms / n;
    printf("%s: %.2f us per launch, %.0f MB written -> %.2f TB/s\n", variant ? "slab + 4 byte gathers per lane" : "slab only",
           us, out_bytes / 1e6, out_bytes / (us * 1e-6) / 1e12);
  }
  (void)hipFree(out);
  (void)hipFree(img);
  return 0;
}
