// CU-mask semantics on gfx950 (hipExtStreamCreateWithCUMask): for each mask,
// run 8192 one-wave blocks (each spinning ~20 us so that every available CU is
// used) and count the distinct (XCC, SE, SH, CU) that ran them, per XCC.
//   hipcc --offload-arch=gfx950 -O2 -o tools/cumask_probe2.bin tools/cumask_probe2.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <set>
#include <string>
#include <vector>

__global__ void k_where(unsigned* out) {
    if (threadIdx.x == 0) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < 2000) {}  // ~20 us at 100 MHz
}

static void run(const char* name, const std::vector<uint32_t>& mask, unsigned* d, int nblk) {
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
        printf("%s: stream creation failed\n", name);
        return;
    }
    hipLaunchKernelGGL(k_where, dim3(nblk), dim3(64), 0, s, d);
    if (hipStreamSynchronize(s) != hipSuccess) { printf("%s: failed\n", name); return; }
    std::vector<unsigned> h(2 * nblk);
    if (hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess) return;
    std::set<unsigned> all;
    int per[8] = {0};
    std::set<unsigned> perx[8];
    for (int i = 0; i < nblk; i++) {
        const unsigned x = h[2 * i] & 7, hw = h[2 * i + 1];
        const unsigned id = ((hw >> 13) & 7) * 64 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 15);
        perx[x].insert(id);
        all.insert(x * 1024 + id);
    }
    printf("%-28s distinct CUs %3zu; per XCC:", name, all.size());
    for (int x = 0; x < 8; x++) printf(" %zu", perx[x].size());
    printf("\n");
    hipStreamDestroy(s);
}

int main() {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    const int nblk = 8192;
    unsigned* d;
    if (hipMalloc(&d, 2 * nblk * sizeof(unsigned)) != hipSuccess) return 1;
    const int nw = (ncu + 31) / 32;
    auto full = [&] { std::vector<uint32_t> m(nw, 0xffffffffu); if (ncu % 32) m[nw - 1] = (1u << (ncu % 32)) - 1; return m; };
    run("full", full(), d, nblk);
    auto without = [&](std::vector<int> bits) { auto m = full(); for (int b : bits) m[b / 32] &= ~(1u << (b % 32)); return m; };
    run("-bit255", without({255}), d, nblk);
    run("-bit0", without({0}), d, nblk);
    run("-bits248..255", without({248, 249, 250, 251, 252, 253, 254, 255}), d, nblk);
    run("-bits0..7", without({0, 1, 2, 3, 4, 5, 6, 7}), d, nblk);
    run("-bits{31,63,..,255}", without({31, 63, 95, 127, 159, 191, 223, 255}), d, nblk);
    run("-bits{7,15,..,63}", without({7, 15, 23, 31, 39, 47, 55, 63}), d, nblk);
    run("-word0 (bits 0..31)", without({0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,24,25,26,27,28,29,30,31}), d, nblk);
    hipFree(d);
    return 0;
}
