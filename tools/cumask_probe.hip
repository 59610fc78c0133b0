// Which XCD / CU does bit i of a stream CU mask (hipExtStreamCreateWithCUMask)
// select?  For each probed bit: a stream masked to that one CU runs 64 blocks,
// each recording HW_REG_XCC_ID and HW_REG_HW_ID; prints the distinct values.
//   hipcc --offload-arch=gfx950 -O2 -o tools/cumask_probe.bin tools/cumask_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <set>
#include <vector>

__global__ void k_where(unsigned* out) {
    if (threadIdx.x == 0) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int ncu = p.multiProcessorCount;
    printf("CUs %d\n", ncu);
    unsigned* d;
    hipMalloc(&d, 2 * 64 * sizeof(unsigned));
    const int bits[] = {0, 1, 2, 3, 7, 8, 9, 31, 32, 63, 64, 128, 248, 249, 255};
    for (int b : bits) {
        if (b >= ncu) continue;
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        mask[b / 32] = 1u << (b % 32);
        hipStream_t s;
        if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
            printf("bit %d: stream creation failed\n", b);
            continue;
        }
        hipLaunchKernelGGL(k_where, dim3(64), dim3(64), 0, s, d);
        hipStreamSynchronize(s);
        std::vector<unsigned> h(128);
        hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
        std::set<unsigned> xs, cus;
        for (int i = 0; i < 64; i++) {
            xs.insert(h[2 * i]);
            const unsigned hw = h[2 * i + 1];
            // HW_ID: wave 3:0, simd 5:4, pipe 7:6, cu 11:8, sh 12, se 15:13 (gfx9 layout)
            cus.insert(((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 20 + ((hw >> 8) & 15));
        }
        printf("bit %3d: xcc", b);
        for (unsigned x : xs) printf(" %u", x);
        printf(" | se*100+sh*20+cu");
        for (unsigned c : cus) printf(" %u", c);
        printf("\n");
        hipStreamDestroy(s);
    }
    hipFree(d);
    return 0;
}
