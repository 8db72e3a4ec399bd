// Block-A microbenchmark: the forward's S phase in isolation (32 v_mfma_f32_32x32x16_bf16 over 16 K fragments read
// from the swizzled LDS image), one wave per SIMD, 4 waves per CU, cycles per block by s_memtime. Variants:
//   0: as variant 11 (S in VGPRs "+v", Q in AGPRs "a", K by ds_read_b128, per-fragment rolling ring)
//   1: 0 without the LDS reads (K fragments held in registers)
//   2: 0 with S in the accumulator file ("+a") and Q in VGPRs
//   3: 1 with S in the accumulator file
//   4: 0 + 8 LDS-DMA pieces (1 KiB each) per wave issued at the block start, landing inside the block
//   5: 0 + the same 8 pieces issued right after the block, landing at the start of the next one
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form tools/r5/mfma_lds_micro.hip -o mfma_lds_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}
__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
template <int OFF>
__device__ __forceinline__ bf16x8 rd(uint32_t a) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF) : "memory");
  return r;
}
template <int N>
__device__ __forceinline__ void wait_tie(bf16x8& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <bool ACC>
__device__ __forceinline__ void mf_first(f32x16& s, const bf16x8& k, const bf16x8& q) {
  if constexpr (ACC)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&a"(s) : "v"(k), "v"(q));
  else
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(s) : "v"(k), "a"(q));
}
template <bool ACC>
__device__ __forceinline__ void mf(f32x16& s, const bf16x8& k, const bf16x8& q) {
  if constexpr (ACC)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(s) : "v"(k), "v"(q));
  else
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(s) : "v"(k), "a"(q));
}

template <int VAR>
__global__ __launch_bounds__(256) void micro(const bf16x8* __restrict__ src, float* __restrict__ out,
                                             unsigned long long* __restrict__ cyc, int iters) {
  constexpr bool LDS = VAR != 1 && VAR != 3, ACC = VAR == 2 || VAR == 3;
  constexpr bool DMA_IN = VAR == 4, DMA_AFTER = VAR == 5;
  const int w = threadIdx.x >> 6;
  __shared__ __attribute__((aligned(1024))) char smem[96 * 1024];  // 1 workgroup per CU, as the forward
  const int lane = threadIdx.x & 63, h = lane >> 5;
  for (int i = threadIdx.x; i < 96 * 1024 / 16; i += 256)
    reinterpret_cast<bf16x8*>(smem)[i] = src[(i + blockIdx.x) & 4095];
  __syncthreads();
  bf16x8 qf[2][8];
  for (int qh = 0; qh < 2; ++qh)
    for (int ks = 0; ks < 8; ++ks) qf[qh][ks] = src[(lane * 16 + qh * 8 + ks + threadIdx.x) & 4095];
  const int row = lane & 31;
  const uint32_t P0 = (uint32_t)(uintptr_t)smem + (uint32_t)(row * 256) + 16u * (uint32_t)(h ^ swz(row));
  uint32_t ak[8];
  for (int ks = 0; ks < 8; ++ks) ak[ks] = P0 ^ (32u * ks);
  bf16x8 kreg[2][4];
  for (int b = 0; b < 2; ++b)
    for (int i = 0; i < 4; ++i) kreg[b][i] = src[(lane * 8 + 4 * b + i) & 4095];
  f32x16 sn[2][2];
  float acc = 0.f;
  unsigned long long total = 0;
  for (int it = 0; it < iters; ++it) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    auto dma = [&]() {
      for (int j = 0; j < 8; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(src + ((lane + 64 * (8 * w + j) + 512 * (it & 1)) & 4095)),
                                         (__attribute__((address_space(3))) void*)(smem + 32768 + (8 * w + j) * 1024),
                                         16, 0, 0);
    };
    if constexpr (DMA_IN) dma();
    bf16x8 kr[2][4];
    auto rdg = [&](auto GC, auto IC) {
      constexpr int g = decltype(GC)::value, i = decltype(IC)::value, t = g >> 1, j = g & 1;
      if constexpr (LDS) kr[g & 1][i] = rd<8192 * t>(ak[4 * j + i]);
    };
    if constexpr (!LDS) {
      sfor<0, 4>([&](auto IC) { kr[0][IC] = kreg[0][IC]; kr[1][IC] = kreg[1][IC]; });
    }
    sfor<0, 4>([&](auto IC) { rdg(std::integral_constant<int, 0>{}, IC); });
    sfor<0, 4>([&](auto IC) { rdg(std::integral_constant<int, 1>{}, IC); });
    sfor<0, 4>([&](auto GC) {
      constexpr int g = decltype(GC)::value, t = g >> 1, j = g & 1, b = g & 1;
      sfor<0, 4>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        constexpr int after = g < 2 ? 7 : (g == 2 ? 7 - i : 3 - i);
        if constexpr (LDS) wait_tie<after>(kr[b][i]);
        sfor<0, 2>([&](auto QC) {
          constexpr int qh = decltype(QC)::value;
          if constexpr (j == 0 && i == 0)
            mf_first<ACC>(sn[t][qh], kr[b][i], qf[qh][4 * j + i]);
          else
            mf<ACC>(sn[t][qh], kr[b][i], qf[qh][4 * j + i]);
          __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr (g < 2) rdg(std::integral_constant<int, g + 2>{}, IC);
      });
    });
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 3" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (DMA_AFTER) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      dma();
    }
    if constexpr (DMA_IN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    total += t1 - t0;
    acc += sn[0][0][it & 15] + sn[1][1][(it + 3) & 15];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (lane == 0) atomicAdd(cyc, total);
}

int main() {
  const int nwg = 1024, iters = 2000;
  std::vector<uint16_t> host(4096 * 8);
  uint32_t x = 12345;
  for (auto& v : host) {
    x = x * 1664525u + 1013904223u;
    v = (uint16_t)(0x3c00 | ((x >> 16) & 0x7f) | (((x >> 24) & 1) << 15));  // bf16 in [-1.99, -1] U [1, 1.99]
  }
  bf16x8* src;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&src, host.size() * 2);
  hipMalloc(&out, nwg * 256 * 4);
  hipMalloc(&cyc, 8);
  hipMemcpy(src, host.data(), host.size() * 2, hipMemcpyHostToDevice);
  auto run = [&](int var) {
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(cyc, 0, 8);
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      switch (var) {
        case 0: micro<0><<<nwg, 256>>>(src, out, cyc, iters); break;
        case 1: micro<1><<<nwg, 256>>>(src, out, cyc, iters); break;
        case 2: micro<2><<<nwg, 256>>>(src, out, cyc, iters); break;
        case 3: micro<3><<<nwg, 256>>>(src, out, cyc, iters); break;
        case 4: micro<4><<<nwg, 256>>>(src, out, cyc, iters); break;
        case 5: micro<5><<<nwg, 256>>>(src, out, cyc, iters); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      const double per = (double)c / (nwg * 4.0 * iters);
      printf("variant %d rep %d: %.1f cycles per block (%.2f per MFMA), %.3f ms, %.0f TF/s\n", var, rep, per, per / 32,
             ms, 2.0 * 32 * 32 * 16 * 32 * nwg * 4.0 * iters / (ms * 1e-3) / 1e12);
    }
  };
  for (int v = 0; v < 6; ++v) run(v);
  return 0;
}
