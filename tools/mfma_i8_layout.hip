// Probe of the operand layout of v_mfma_i32_32x32x32_i8 / 16x16x64_i8 on gfx950: each lane's
// raw fragments in, the raw accumulators out (tools/mfma_i8_layout.py checks layout hypotheses
// against a CPU matmul with exact integer data).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_i8_layout tools/mfma_i8_layout.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k32(const int *a, const int *b, int *d) {
    const int l = threadIdx.x;
    v4i A = {a[4 * l], a[4 * l + 1], a[4 * l + 2], a[4 * l + 3]};
    v4i B = {b[4 * l], b[4 * l + 1], b[4 * l + 2], b[4 * l + 3]};
    v16i C = {0};
    C = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, C, 0, 0, 0);
    for (int r = 0; r < 16; ++r) d[16 * l + r] = C[r];
}

__global__ void k16(const int *a, const int *b, int *d) {
    const int l = threadIdx.x;
    v4i A = {a[4 * l], a[4 * l + 1], a[4 * l + 2], a[4 * l + 3]};
    v4i B = {b[4 * l], b[4 * l + 1], b[4 * l + 2], b[4 * l + 3]};
    v4i C = {0, 0, 0, 0};
    C = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B, C, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[4 * l + r] = C[r];
}

int main() {
    int ha[256], hb[256], hd[1024];
    srand(7);
    for (int i = 0; i < 256; ++i) {
        ha[i] = rand();
        hb[i] = rand();
    }
    int *da, *db, *dd;
    hipMalloc(&da, 1024);
    hipMalloc(&db, 1024);
    hipMalloc(&dd, 4096);
    hipMemcpy(da, ha, 1024, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, 1024, hipMemcpyHostToDevice);
    k32<<<1, 64>>>(da, db, dd);
    hipMemcpy(hd, dd, 4096, hipMemcpyDeviceToHost);
    printf("{\"a\": [");
    for (int i = 0; i < 256; ++i) printf("%s%d", i ? "," : "", ha[i]);
    printf("], \"b\": [");
    for (int i = 0; i < 256; ++i) printf("%s%d", i ? "," : "", hb[i]);
    printf("], \"d32\": [");
    for (int i = 0; i < 1024; ++i) printf("%s%d", i ? "," : "", hd[i]);
    k16<<<1, 64>>>(da, db, dd);
    hipMemcpy(hd, dd, 1024, hipMemcpyDeviceToHost);
    printf("], \"d16\": [");
    for (int i = 0; i < 256; ++i) printf("%s%d", i ? "," : "", hd[i]);
    printf("]}\n");
    return 0;
}
