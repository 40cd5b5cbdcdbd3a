// Probe: which XCD (HW_REG_XCC_ID) and CU each workgroup of a launch runs on, to check the
// blockIdx -> XCD dealing the tile orderings assume (blockIdx % 8). One launch of B
// workgroups of 256 threads; prints the XCD histogram of blockIdx % 8 classes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void probe(unsigned* out) {
    if (threadIdx.x == 0) {
        // s_getreg_b32 HW_REG_XCC_ID (id 20), bits [3:0]: simm16 = (size-1) << 11 | offset << 6 | id
        const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
        // HW_REG_HW_ID (id 4): CU_ID bits [11:8], SH_ID [12], SE_ID [15:13]
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
    // keep the workgroup alive a little so dispatch spreads
    for (volatile int i = 0; i < 2000; ++i) {}
}

int main() {
    const int B = 4096;
    unsigned* d;
    CK(hipMalloc(&d, 2 * B * sizeof(unsigned)));
    probe<<<B, 256>>>(d);
    CK(hipDeviceSynchronize());
    std::vector<unsigned> h(2 * B);
    CK(hipMemcpy(h.data(), d, 2 * B * sizeof(unsigned), hipMemcpyDeviceToHost));
    int hist[8][8] = {};
    for (int b = 0; b < B; ++b) hist[b % 8][h[2 * b] & 7]++;
    printf("rows: blockIdx %% 8, cols: XCC id\n");
    for (int r = 0; r < 8; ++r) {
        printf("%d:", r);
        for (int c = 0; c < 8; ++c) printf(" %5d", hist[r][c]);
        printf("\n");
    }
    printf("first 24 blocks xcc: ");
    for (int b = 0; b < 24; ++b) printf("%u ", h[2 * b] & 7);
    printf("\n");
    return 0;
}
