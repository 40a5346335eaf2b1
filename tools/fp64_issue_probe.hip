// fp64_issue_probe.hip -- per-SIMD f64 issue behaviour on gfx950 (diagnostic for the blind-rotate
// kernels): cycles per v_fma_f64 for C independent chains per wave at W waves per SIMD, one
// workgroup per CU, s_memtime around the loop (median over workgroups).  Also 32-bit DPP moves and
// v_permlane32_swap streams beside f64 work.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

template <int C>
__global__ void k_fma(unsigned long long* cyc, double* out, double a, double b, int iters) {
    double x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = threadIdx.x + c;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 32 / C; ++k)
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = __fma_rn(x[c], a, b);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int C>
__global__ void k_fma_dpp(unsigned long long* cyc, double* out, double a, double b, int iters) {
    // C f64 chains plus, per 32 fmas, 16 DPP moves (the bank-masked transposes' shape)
    double x[C];
    int y[4] = {(int)threadIdx.x, 1, 2, 3};
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = threadIdx.x + c;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 32 / C; ++k) {
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = __fma_rn(x[c], a, b);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int d = 0; d < 4; ++d) y[d] = __builtin_amdgcn_update_dpp(y[d], y[(d + 1) & 3], 0x118, 0xF, 0xC, false);
    }
    double s = y[0] + y[1] + y[2] + y[3];
#pragma unroll
    for (int c = 0; c < C; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int C>
__global__ void k_add32(unsigned long long* cyc, double* out, double a, double b, int iters) {
    // C independent 32-bit integer chains (v_add_u32 / v_xor), the transposes' and index math's class
    uint32_t x[C];
    const uint32_t ia = (uint32_t)(a * 1000.0), ib = (uint32_t)(b * 1e9);
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = threadIdx.x + c;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 32 / C; ++k)
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = (x[c] + ia) ^ ib;
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
double run(K kern, int waves_per_simd, int iters, const char* name, int ops_per_iter) {
    const int blocks = 256, threads = 256 * waves_per_simd;
    unsigned long long* c; double* d;
    hipMalloc(&c, blocks * 8); hipMalloc(&d, (size_t)blocks * threads * 8);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, c, d, 0.999999, 1e-7, 8);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, c, d, 0.999999, 1e-7, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(blocks);
    hipMemcpy(h.data(), c, blocks * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    const double per = (double)h[blocks / 2] / ((double)iters * ops_per_iter);  // cycles per op per wave
    const double tflops = 2.0 * ops_per_iter * (double)iters * blocks * threads / (ms * 1e-3) / 1e12;
    printf("%-28s waves/SIMD %d: %.2f ticks per op per wave -> %.2f per op per SIMD; kernel %.3f ms, %.1f TF/s f64 fma, "
           "%.2f ticks/ns\n", name, waves_per_simd, per, per / waves_per_simd, ms, tflops, (double)h[blocks / 2] / (ms * 1e6));
    hipFree(c); hipFree(d);
    return per;
}

int main() {
    for (int w : {1, 2, 3, 4}) {
        run(k_fma<1>, w, 512, "fma_f64 1 chain", 32);
        run(k_fma<2>, w, 512, "fma_f64 2 chains", 32);
        run(k_fma<4>, w, 512, "fma_f64 4 chains", 32);
        run(k_fma<8>, w, 512, "fma_f64 8 chains", 32);
        run(k_fma_dpp<8>, w, 512, "fma_f64 8 chains + 16 dpp", 32);
        run(k_add32<8>, w, 512, "add+xor u32 8 chains", 64);
    }
    return 0;
}
