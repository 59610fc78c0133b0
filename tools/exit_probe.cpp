// Process exit cost after HIP use (tests/example wall):
//   exit_probe MODE   prints the epoch ms just before _exit(0)
// MODE 0: no HIP; 1: HIP runtime (psx_device_count); 2: + psx_warmup_for(0, 2, 0)
// (context + code objects of a c = 2 run); 3: + psx_warmup(0) (all code objects);
// 4: + a 256 MB device buffer (hipMalloc'd through the engine: one exhaustive
// c = 2 pass on a tiny locus is not needed, the allocation is what is timed).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <unistd.h>

#include "../include/pipsort_engine.h"

static double epoch_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::system_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const double t0 = epoch_ms();
    int nd = 0;
    if (mode >= 1) psx_device_count(&nd);
    const double t1 = epoch_ms();
    if (mode == 2) psx_warmup_for(0, 2, 0);
    if (mode >= 3) psx_warmup(0);
    const double t2 = epoch_ms();
    printf("{\"mode\": %d, \"runtime_ms\": %.3f, \"warm_ms\": %.3f, \"exit_epoch_ms\": %.3f}\n", mode, t1 - t0, t2 - t1,
           epoch_ms());
    fflush(stdout);
    _exit(0);
}
