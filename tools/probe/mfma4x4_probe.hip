// Layout probe for v_mfma_f32_4x4x1_16b_f32 (gfx950) and an fmaf-chain check of
// v_mfma_f32_16x16x4_f32 (tools only; run once on the GPU, results in profiles/).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k_probe(const float* a, const float* b, float* d) {
    const int l = threadIdx.x;
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a[l], b[l], c, 0, 0, 0);
    for (int j = 0; j < 4; ++j) d[l * 4 + j] = c[j];
}
// 16x16x4 f32: A[i][k] from lane i + 16k, B[k][j] from lane j + 16k; D[i][j]: lane j + 16*(i/4), reg i%4
__global__ void k_chain(const float* a, const float* b, const float* c0, float* d, float* e) {
    const int l = threadIdx.x;
    f32x4 c = {c0[l * 4], c0[l * 4 + 1], c0[l * 4 + 2], c0[l * 4 + 3]};
    f32x4 r = __builtin_amdgcn_mfma_f32_16x16x4f32(a[l], b[l], c, 0, 0, 0);
    for (int j = 0; j < 4; ++j) d[l * 4 + j] = r[j];
    // the same as an fmaf chain in k order, for D row i = 4*(l>>4)+j, col = l&15
    for (int j = 0; j < 4; ++j) {
        const int i = 4 * (l >> 4) + j, col = l & 15;
        float acc = c[j];
        for (int k = 0; k < 4; ++k) acc = fmaf(a[i + 16 * k], b[col + 16 * k], acc);
        e[l * 4 + j] = acc;
    }
}
int main() {
    float *a, *b, *c, *d, *e;
    hipMalloc(&a, 256); hipMalloc(&b, 256); hipMalloc(&c, 1024); hipMalloc(&d, 1024); hipMalloc(&e, 1024);
    float ha[64], hb[64], hd[256], he[256], hc[256];
    // run 1: A = lane + 1, B = 1 -> D[r][c] names the lane that supplies row r
    for (int i = 0; i < 64; ++i) { ha[i] = i + 1; hb[i] = 1; }
    hipMemcpy(a, ha, 256, hipMemcpyHostToDevice); hipMemcpy(b, hb, 256, hipMemcpyHostToDevice);
    k_probe<<<1, 64>>>(a, b, d); hipMemcpy(hd, d, 1024, hipMemcpyDeviceToHost);
    printf("4x4x1_16b A-lane (row provider) per (lane, reg):\n");
    for (int l = 0; l < 16; ++l) printf("lane %2d: %g %g %g %g\n", l, hd[4*l]-1, hd[4*l+1]-1, hd[4*l+2]-1, hd[4*l+3]-1);
    // run 2: A = 1, B = lane + 1 -> names the lane that supplies column c
    for (int i = 0; i < 64; ++i) { ha[i] = 1; hb[i] = i + 1; }
    hipMemcpy(a, ha, 256, hipMemcpyHostToDevice); hipMemcpy(b, hb, 256, hipMemcpyHostToDevice);
    k_probe<<<1, 64>>>(a, b, d); hipMemcpy(hd, d, 1024, hipMemcpyDeviceToHost);
    printf("4x4x1_16b B-lane (col provider) per (lane, reg):\n");
    for (int l = 0; l < 16; ++l) printf("lane %2d: %g %g %g %g\n", l, hd[4*l]-1, hd[4*l+1]-1, hd[4*l+2]-1, hd[4*l+3]-1);
    // chain check on random data with cancellation
    srand(1);
    long bad = 0, tot = 0;
    for (int it = 0; it < 20000; ++it) {
        for (int i = 0; i < 64; ++i) {
            ha[i] = (float)(rand() - RAND_MAX / 2) / (float)(rand() % 1000 + 1) * 1e-3f * (float)(1 << (rand() % 20));
            hb[i] = (float)(rand() - RAND_MAX / 2) / (float)(rand() % 1000 + 1) * 1e-3f;
        }
        for (int i = 0; i < 256; ++i) hc[i] = (float)(rand() - RAND_MAX / 2) / (float)(rand() % 1000 + 1);
        hipMemcpy(a, ha, 256, hipMemcpyHostToDevice); hipMemcpy(b, hb, 256, hipMemcpyHostToDevice);
        hipMemcpy(c, hc, 1024, hipMemcpyHostToDevice);
        k_chain<<<1, 64>>>(a, b, c, d, e);
        hipMemcpy(hd, d, 1024, hipMemcpyDeviceToHost); hipMemcpy(he, e, 1024, hipMemcpyDeviceToHost);
        for (int i = 0; i < 256; ++i) { ++tot; if (memcmp(&hd[i], &he[i], 4)) ++bad; }
    }
    printf("16x16x4 f32 vs fmaf chain in k order: %ld of %ld differ\n", bad, tot);
    return 0;
}
