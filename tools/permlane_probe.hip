// v_permlane{16,32}_swap(v, v) lane mapping on the device: prints, per lane, the two results
// for v = lane (the screen's xor32_f relies on lane < 32 -> second result = lane + 32).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *o) {
    const unsigned v = threadIdx.x;
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    const auto q = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    o[4 * v] = p[0]; o[4 * v + 1] = p[1]; o[4 * v + 2] = q[0]; o[4 * v + 3] = q[1];
}
int main() {
    unsigned *d, h[256];
    hipMalloc(&d, 1024);
    k<<<1, 64>>>(d);
    hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; l++) {
        if ((l < 32 ? h[4 * l + 1] : h[4 * l]) != (unsigned)(l ^ 32)) bad++;
        const unsigned a = h[4 * l + 2], b = h[4 * l + 3];
        if (!((a == (unsigned)l && b == (unsigned)(l ^ 16)) || (b == (unsigned)l && a == (unsigned)(l ^ 16)))) bad++;
    }
    for (int l = 0; l < 64; l += 15) printf("lane %d: p32 %u %u p16 %u %u\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
    printf("permlane probe: %s\n", bad ? "MISMATCH" : "ok");
    return bad ? 1 : 0;
}
