// Operand-map probe for v_mfma_i32_16x16x64_i8 on gfx950 (MI355X_MICROARCH/cdna_hip_programming:
// "check the map with exact integer data").  Random int8 fragments in, C out; the host tests the
// candidate k-maps and prints the one that reproduces C exactly.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void probe(const v4i* a, const v4i* b, v4i* d) {
    const int l = threadIdx.x;
    v4i acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[l], b[l], acc, 0, 0, 0);
    d[l] = acc;
}

int main() {
    int8_t ha[64][16], hb[64][16];
    int hd[64][4];
    srand(7);
    for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 16; ++j) {
            ha[l][j] = (int8_t)(rand() % 255 - 127);
            hb[l][j] = (int8_t)(rand() % 255 - 127);
        }
    v4i *da, *db, *dd;
    hipMalloc(&da, 1024); hipMalloc(&db, 1024); hipMalloc(&dd, 1024);
    hipMemcpy(da, ha, 1024, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, dd);
    hipMemcpy(hd, dd, 1024, hipMemcpyDeviceToHost);
    // candidate maps: lane l, byte j -> k
    const char* names[2] = {"k = 16(l>>4) + j", "k = 8(l>>4) + j (j<8), 32 + 8(l>>4) + j-8 (j>=8)"};
    for (int m = 0; m < 2; ++m) {
        int8_t A[16][64], B[64][16];
        for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 16; ++j) {
                int k = m == 0 ? 16 * (l >> 4) + j : (j < 8 ? 8 * (l >> 4) + j : 32 + 8 * (l >> 4) + j - 8);
                A[l & 15][k] = ha[l][j];
                B[k][l & 15] = hb[l][j];
            }
        int bad = 0;
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 4; ++r) {
                int row = (l >> 4) * 4 + r, col = l & 15;
                long s = 0;
                for (int k = 0; k < 64; ++k) s += (long)A[row][k] * B[k][col];
                if (s != hd[l][r]) ++bad;
            }
        printf("map %d (%s): %d mismatches of 256\n", m, names[m], bad);
    }
    return 0;
}
