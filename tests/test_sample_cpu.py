"""psx::discrete_draw (pipsort_amd/csrc/psx_sample.h), the SSS walk's neighbour
draw, against libstdc++'s std::discrete_distribution, which the reference
calls (sss_postcal.cpp:296-343): the same index for every draw and the same
generator state afterwards, on weight vectors of the walk's kind (exp(lk - max)
with ties, zeros, underflow, one and two entries)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HARNESS = r"""
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>
#include "psx_sample.h"

int main() {
    std::mt19937 wgen(7);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::mt19937 ga(12345), gb(12345);
    const size_t sizes[] = {1, 2, 3, 4, 17, 200, 975, 1000, 4096};
    long draws = 0, bad = 0;
    for (int rep = 0; rep < 400; rep++) {
        for (size_t n : sizes) {
            std::vector<double> lk(n);
            const int kind = rep % 5;
            for (size_t i = 0; i < n; i++) {
                double x = -U(wgen) * (kind == 0 ? 5.0 : kind == 1 ? 50.0 : 800.0);
                if (kind == 3 && i % 3 == 0) x = 0.0;             // ties at the max
                if (kind == 4 && i % 2 == 1) x = -1e308;          // exact zeros after exp
                lk[i] = x;
            }
            const double mx = *std::max_element(lk.begin(), lk.end());
            std::vector<double> pr(n);
            double s = 0.0;
            for (size_t i = 0; i < n; i++) s += (pr[i] = std::exp(lk[i] - mx));
            std::discrete_distribution<size_t> dist(pr.begin(), pr.end());
            for (int d = 0; d < 5; d++) {
                const size_t a = dist(ga);
                const size_t b = psx::discrete_draw(pr.data(), n, s, gb);
                draws++;
                if (a != b) bad++;
            }
            if (std::accumulate(pr.begin(), pr.end(), 0.0) != s) bad++;
        }
    }
    const bool same_state = ga == gb;
    std::printf("%ld %ld %d\n", draws, bad, same_state ? 1 : 0);
    return 0;
}
"""


CLANG = "/opt/rocm/llvm/bin/clang++"  # hipcc's host compiler (the engine's host code)


@pytest.mark.parametrize("cxx", [["g++", "-O2"], [CLANG, "-O3"]], ids=["gcc", "rocm-clang"])
def test_discrete_draw_matches_libstdcxx(tmp_path, cxx):
    if not os.path.exists(cxx[0]) and os.sep in cxx[0]:
        pytest.skip(f"{cxx[0]} absent")
    src = tmp_path / "h.cpp"
    src.write_text(HARNESS)
    exe = tmp_path / "h"
    r = subprocess.run(cxx + ["-std=c++17", "-I", os.path.join(ROOT, "pipsort_amd", "csrc"), str(src),
                              "-o", str(exe)], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail(r.stderr)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    draws, bad, same_state = int(out[0]), int(out[1]), int(out[2])
    assert draws == 400 * 9 * 5
    assert bad == 0
    assert same_state == 1
