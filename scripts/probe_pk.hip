// Issue-rate probe (gfx950): v_fma_f32 vs v_pk_fma_f32 vs v_exp_f32 chains, 8 independent accumulators per lane,
// W waves per SIMD. Prints ns per wave-instruction per SIMD. Build: hipcc --offload-arch=gfx950 -O3 probe_pk.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

__global__ void k_fma(float *out, float a, float b) {
    float x[8];
    for (int j = 0; j < 8; j++) x[j] = threadIdx.x + j;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = __builtin_fmaf(x[j], a, b);
    float s = 0;
    for (int j = 0; j < 8; j++) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_pkfma(float *out, float a, float b) {
    f2 x[8];
    const f2 av = {a, a}, bv = {b, b};
    for (int j = 0; j < 8; j++) x[j] = f2{(float)threadIdx.x + j, (float)j};
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = __builtin_elementwise_fma(x[j], av, bv);
    float s = 0;
    for (int j = 0; j < 8; j++) s += x[j].x + x[j].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_exp(float *out, float a, float b) {
    float x[8];
    for (int j = 0; j < 8; j++) x[j] = (threadIdx.x + j) * 1e-3f;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = __builtin_amdgcn_exp2f(x[j]) * a;  // exp + mul
    float s = 0;
    for (int j = 0; j < 8; j++) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    float *out;
    hipMalloc(&out, 256 * 8 * 256 * sizeof(float) * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 1; w <= 8; w *= 2) {  // waves per SIMD: w * 4 waves per CU = w blocks of 256 threads per CU
        const int blocks = 256 * w;
        const char *names[3] = {"v_fma_f32", "v_pk_fma_f32", "v_exp_f32+v_mul"};
        for (int k = 0; k < 3; k++) {
            for (int rep = 0; rep < 2; rep++) {
                hipEventRecord(e0);
                if (k == 0) k_fma<<<blocks, 256>>>(out, 0.999f, 0.001f);
                if (k == 1) k_pkfma<<<blocks, 256>>>(out, 0.999f, 0.001f);
                if (k == 2) k_exp<<<blocks, 256>>>(out, 0.5f, 0.f);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                // wave-instructions per SIMD in the loop: w waves x ITERS x 8
                const double winst = (double)w * ITERS * 8;
                if (rep) printf("waves/SIMD %d  %-16s %.3f ms  %.3f ns per wave-instr per SIMD\n", w, names[k], ms,
                                ms * 1e6 / winst);
            }
        }
    }
    hipFree(out);
    return 0;
}
