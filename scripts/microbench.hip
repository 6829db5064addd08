// microbench.hip — gfx950 throughput of the instructions the tone-map kernel
// is made of.  Each kernel runs 8 independent dependency chains per lane,
// 2048 blocks x 256 threads (8 waves / SIMD), and reports wave-instructions
// per clock per CU (clock from GRBM-free estimate: 2.4 GHz nominal) and the
// cost relative to v_fma_f32.
//   hipcc --offload-arch=gfx950 -O3 scripts/microbench.hip -o /tmp/mb && /tmp/mb
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define ITERS 2048
#define CHK(x)                                                          \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);  \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

#define CHAIN8(INSTR)                                          \
  asm volatile(INSTR : "+v"(x0));                              \
  asm volatile(INSTR : "+v"(x1));                              \
  asm volatile(INSTR : "+v"(x2));                              \
  asm volatile(INSTR : "+v"(x3));                              \
  asm volatile(INSTR : "+v"(x4));                              \
  asm volatile(INSTR : "+v"(x5));                              \
  asm volatile(INSTR : "+v"(x6));                              \
  asm volatile(INSTR : "+v"(x7));

#define UNARY_KERNEL(NAME, INSTR)                                                          \
  __global__ __launch_bounds__(256) void NAME(float* out, float seed) {                   \
    float x0 = seed + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,    \
          x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                                           \
    for (int i = 0; i < ITERS; i++) {                                                      \
      CHAIN8(INSTR)                                                                        \
    }                                                                                      \
    out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;           \
  }

UNARY_KERNEL(k_fma, "v_fma_f32 %0, %0, %0, 1.0")
UNARY_KERNEL(k_mul, "v_mul_f32 %0, %0, 0.5")
UNARY_KERNEL(k_exp, "v_exp_f32 %0, %0")
UNARY_KERNEL(k_log, "v_log_f32 %0, %0")
UNARY_KERNEL(k_rcp, "v_rcp_f32 %0, %0")
UNARY_KERNEL(k_sqrt, "v_sqrt_f32 %0, %0")
UNARY_KERNEL(k_fract, "v_fract_f32 %0, %0")
UNARY_KERNEL(k_cvt, "v_cvt_i32_f32 %0, %0")
UNARY_KERNEL(k_med3, "v_med3_f32 %0, %0, 0, 1.0")
UNARY_KERNEL(k_pkfma16, "v_pk_fma_f16 %0, %0, %0, %0")
UNARY_KERNEL(k_mad24, "v_mad_u32_u24 %0, %0, 7, %0")
UNARY_KERNEL(k_fmac, "v_fmac_f32 %0, %0, %0")
UNARY_KERNEL(k_add, "v_add_f32 %0, %0, %0")
UNARY_KERNEL(k_max, "v_max_f32 %0, %0, 1.0")
UNARY_KERNEL(k_min, "v_min_f32 %0, %0, 1.0")
UNARY_KERNEL(k_max3, "v_max3_f32 %0, %0, 1.0, %0")

UNARY_KERNEL(k_addu, "v_add_u32 %0, 7, %0")
UNARY_KERNEL(k_lsh, "v_lshlrev_b32 %0, 1, %0")
UNARY_KERNEL(k_and, "v_and_b32 %0, 7, %0")
UNARY_KERNEL(k_mov, "v_mov_b32 %0, 1.0")
UNARY_KERNEL(k_movdpp, "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
UNARY_KERNEL(k_adddpp, "v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
UNARY_KERNEL(k_floor, "v_floor_f32 %0, %0")
UNARY_KERNEL(k_cvtf, "v_cvt_f32_i32 %0, %0")

UNARY_KERNEL(k_fmaak, "v_fmaak_f32 %0, %0, %0, 0x3e000000")
UNARY_KERNEL(k_mulu24, "v_mul_u32_u24 %0, 7, %0")
UNARY_KERNEL(k_mullo, "v_mul_lo_u32 %0, %0, %0")
UNARY_KERNEL(k_lshladd, "v_lshl_add_u32 %0, %0, 2, %0")
UNARY_KERNEL(k_cvtu, "v_cvt_u32_f32 %0, %0")
UNARY_KERNEL(k_cvtflr, "v_cvt_flr_i32_f32 %0, %0")
UNARY_KERNEL(k_bfe, "v_bfe_u32 %0, %0, 4, 8")
UNARY_KERNEL(k_andor, "v_and_or_b32 %0, %0, -16, 5")
UNARY_KERNEL(k_lshl16, "v_lshlrev_b16 %0, 1, %0")

// Instructions that read or write SGPR masks.  Every SGPR operand goes
// through a constraint ("s" input / "=s" output) or a declared clobber
// ("vcc"): an asm statement that names a fixed SGPR pair the compiler does
// not know about can overwrite live state -- round 1's k_cmp64 wrote
// s[0:1], the kernarg pointer on entry, and the final out[] store then
// faulted (HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION).
#define CHAIN8_CNDVCC()                                                            \
  asm volatile("v_cndmask_b32 %0, %0, 1.0, vcc" : "+v"(x0) : : "vcc");           \
  asm volatile("v_cndmask_b32 %0, %0, 1.0, vcc" : "+v"(x1) : : "vcc");           \
  asm volatile("v_cndmask_b32 %0, %0, 1.0, vcc" : "+v"(x2) : : "vcc");           \
  asm volatile("v_cndmask_b32 %0, %0, 1.0, vcc" : "+v"(x3) : : "vcc");           \
  asm volatile("v_cndmask_b32 %0, %0, 1.0, vcc" : "+v"(x4) : : "vcc");           \
  asm volatile("v_cndmask_b32 %0, %0, 1.0, vcc" : "+v"(x5) : : "vcc");           \
  asm volatile("v_cndmask_b32 %0, %0, 1.0, vcc" : "+v"(x6) : : "vcc");           \
  asm volatile("v_cndmask_b32 %0, %0, 1.0, vcc" : "+v"(x7) : : "vcc");
#define CND64(X) asm volatile("v_cndmask_b32_e64 %0, %0, 1.0, %1" : "+v"(X) : "s"(m));
#define CMP64(X) asm volatile("v_cmp_gt_f32_e64 %0, %1, 1.0" : "=s"(m) : "v"(X)); acc ^= m;
#define CMPVCC(X) asm volatile("v_cmp_lt_f32_e32 vcc, 1.0, %0" : : "v"(X) : "vcc");

__global__ __launch_bounds__(256) void k_cnd(float* out, float seed) {
  float x0 = seed + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6,
        x7 = x0 + 7;
  for (int i = 0; i < ITERS; i++) {
    CHAIN8_CNDVCC()
  }
  out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

__global__ __launch_bounds__(256) void k_cnd64(float* out, float seed) {
  float x0 = seed + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6,
        x7 = x0 + 7;
  const unsigned long long m = __builtin_amdgcn_ballot_w64(x0 > 8.0f);  // an SGPR pair the compiler owns
  for (int i = 0; i < ITERS; i++) {
    CND64(x0) CND64(x1) CND64(x2) CND64(x3) CND64(x4) CND64(x5) CND64(x6) CND64(x7)
  }
  out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

// compares: VOPC writing VCC (declared clobber) and VOP3 writing an SGPR pair
// the compiler allocates ("=s"), folded into a scalar so none is dead
__global__ __launch_bounds__(256) void k_cmp(float* out, float seed) {
  const float x0 = seed + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,
              x6 = x0 + 6, x7 = x0 + 7;
  for (int i = 0; i < ITERS; i++) {
    CMPVCC(x0) CMPVCC(x1) CMPVCC(x2) CMPVCC(x3) CMPVCC(x4) CMPVCC(x5) CMPVCC(x6) CMPVCC(x7)
  }
  out[blockIdx.x * 256 + threadIdx.x] = x0;
}

__global__ __launch_bounds__(256) void k_cmp64(float* out, float seed) {
  const float x0 = seed + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,
              x6 = x0 + 6, x7 = x0 + 7;
  unsigned long long m, acc = 0;
  for (int i = 0; i < ITERS; i++) {
    CMP64(x0) CMP64(x1) CMP64(x2) CMP64(x3) CMP64(x4) CMP64(x5) CMP64(x6) CMP64(x7)
  }
  out[blockIdx.x * 256 + threadIdx.x] = x0 + (float)(acc & 1);
}

__global__ __launch_bounds__(256) void k_pkfma32(float* out, float seed) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 x0 = {seed, seed + 1}, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6,
     x7 = x0 + 7;
  for (int i = 0; i < ITERS; i++) {
    CHAIN8("v_pk_fma_f32 %0, %0, %0, %0")
  }
  f2 s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
}

// mixed: 1 transcendental + 3 FMAs per step (does the trans pipe overlap?)
__global__ __launch_bounds__(256) void k_mix13(float* out, float seed) {
  float x0 = seed + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6,
        x7 = x0 + 7;
  for (int i = 0; i < ITERS; i++) {
    CHAIN8("v_exp_f32 %0, %0")
    CHAIN8("v_fma_f32 %0, %0, %0, 1.0")
    CHAIN8("v_fma_f32 %0, %0, %0, 1.0")
    CHAIN8("v_fma_f32 %0, %0, %0, 1.0")
  }
  out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

// LDS gather: 8 independent random ds_read_b64 per step from a 32 KiB table
__global__ __launch_bounds__(256) void k_lds(float* out, float seed) {
  __shared__ float2 tab[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) tab[i] = make_float2(i * 0.001f, seed);
  __syncthreads();
  unsigned h[8];
  for (int k = 0; k < 8; k++) h[k] = (threadIdx.x * 2654435761u + k * 40503u + blockIdx.x) & 4095u;
  float acc = 0;
  for (int i = 0; i < ITERS / 8; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      float2 v = tab[h[k]];
      acc += v.x;
      h[k] = (h[k] + (unsigned)(v.x * 7.0f) + 977u) & 4095u;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// global gather from a 65^3 float4 table (4.4 MB), random or local
template <bool LOCAL>
__global__ __launch_bounds__(256) void k_gather(const float4* __restrict__ tab, float* out, int n) {
  unsigned h[8];
  const unsigned base = (blockIdx.x * 256u + threadIdx.x) * 7u;
  for (int k = 0; k < 8; k++) h[k] = (LOCAL ? (base / 64u * 64u + threadIdx.x % 16u + k) : (base * 2654435761u + k * 40503u)) % n;
  float acc = 0;
  for (int i = 0; i < ITERS / 16; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      float4 v = tab[h[k]];
      acc += v.x + v.w;
      h[k] = LOCAL ? (h[k] + 1u + (unsigned)v.w) % n : (h[k] * 1103515245u + 12345u + (unsigned)v.w) % n;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// streaming copy (HBM ceiling for the same access shape: 16 B/lane in, 16 B/lane out)
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  size_t stride = (size_t)gridDim.x * 256;
  for (; i < n; i += stride) b[i] = a[i];
}

typedef void (*kfn)(float*, float);

static double time_kernel(kfn k, float* out, int blocks) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 0.5f);
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CHK(hipEventRecord(a));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 0.5f);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const int blocks = 2048;  // 256 CUs x 8 blocks of 4 waves = 8 waves / SIMD
  float* out;
  CHK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(float)));
  struct {
    const char* name;
    kfn k;
    double instr_per_iter;  // wave-instructions per iteration per wave
  } cases[] = {
      {"v_fma_f32", k_fma, 8},     {"v_mul_f32", k_mul, 8},     {"v_exp_f32", k_exp, 8},
      {"v_log_f32", k_log, 8},     {"v_rcp_f32", k_rcp, 8},     {"v_sqrt_f32", k_sqrt, 8},
      {"v_fract_f32", k_fract, 8}, {"v_cvt_i32_f32", k_cvt, 8}, {"v_med3_f32", k_med3, 8},
      {"v_pk_fma_f16", k_pkfma16, 8}, {"v_mad_u32_u24", k_mad24, 8}, {"v_pk_fma_f32", k_pkfma32, 8},
      {"mix 1exp+3fma", k_mix13, 32},
      {"v_fmac_f32", k_fmac, 8}, {"v_add_f32", k_add, 8}, {"v_max_f32", k_max, 8}, {"v_min_f32", k_min, 8},
      {"v_max3_f32", k_max3, 8}, {"v_cndmask e32", k_cnd, 8}, {"v_cndmask e64", k_cnd64, 8},
      {"v_cmp e32 (vcc)", k_cmp, 8}, {"v_cmp e64 (sgpr)", k_cmp64, 8},
      {"v_add_u32", k_addu, 8}, {"v_lshlrev_b32", k_lsh, 8}, {"v_and_b32", k_and, 8}, {"v_mov_b32", k_mov, 8},
      {"v_mov_b32_dpp", k_movdpp, 8}, {"v_add_f32_dpp", k_adddpp, 8}, {"v_floor_f32", k_floor, 8},
      {"v_mul_u32_u24", k_mulu24, 8}, {"v_mul_lo_u32", k_mullo, 8}, {"v_lshl_add_u32", k_lshladd, 8},
      {"v_cvt_u32_f32", k_cvtu, 8}, {"v_cvt_flr_i32_f32", k_cvtflr, 8}, {"v_bfe_u32", k_bfe, 8},
      {"v_and_or_b32", k_andor, 8}, {"v_lshlrev_b16", k_lshl16, 8},
  };
  const double waves = blocks * 4.0, cus = 256, clk = 2.4e9;
  double fma_rate = 0;
  printf("%-16s %10s %14s %10s\n", "instr", "ms", "instr/clk/CU", "cost(fma=1)");
  for (auto& c : cases) {
    double ms = time_kernel(c.k, out, blocks);
    double instr = waves * ITERS * c.instr_per_iter;
    double rate = instr / (ms * 1e-3) / cus / clk;
    if (!fma_rate) fma_rate = rate;
    printf("%-16s %10.3f %14.3f %10.2f\n", c.name, ms, rate, fma_rate / rate);
  }
  {
    double ms = time_kernel(k_lds, out, blocks);
    double reads = waves * (ITERS / 8) * 8;
    printf("%-16s %10.3f %14.3f  (ds_read_b64 random + ~4 VALU each)\n", "lds gather", ms,
           reads / (ms * 1e-3) / cus / clk);
  }
  const int n = 65 * 65 * 65;
  float4* tab;
  CHK(hipMalloc(&tab, (size_t)n * sizeof(float4)));
  CHK(hipMemset(tab, 0, (size_t)n * sizeof(float4)));
  for (int loc = 0; loc < 2; loc++) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      CHK(hipEventRecord(a));
      if (loc) hipLaunchKernelGGL((k_gather<true>), dim3(blocks), dim3(256), 0, 0, tab, out, n);
      else hipLaunchKernelGGL((k_gather<false>), dim3(blocks), dim3(256), 0, 0, tab, out, n);
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms;
      CHK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    double loads = waves * (ITERS / 16) * 8;
    printf("%-16s %10.3f %14.3f  (global_load_dwordx4 gathers per clk per CU, 4.4 MB table)\n",
           loc ? "gather local" : "gather random", best, loads / (best * 1e-3) / cus / clk);
  }
  {
    size_t bytes = (size_t)2 << 30;
    uint4 *a, *b;
    CHK(hipMalloc(&a, bytes));
    CHK(hipMalloc(&b, bytes));
    CHK(hipMemset(a, 1, bytes));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, a, b, bytes / 16);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    printf("%-16s %10.3f %14.1f GB/s (read+write)\n", "hbm copy 2GiB", best, 2.0 * bytes / (best * 1e-3) / 1e9);
  }
  return 0;
}
