// psx_sample.h — the SSS walk's neighbour draw (sss_postcal.cpp:296-343) without
// std::discrete_distribution's two vectors.
//
// The reference draws with std::discrete_distribution<size_t>(w.begin(), w.end())
// (gen) under libstdc++ (bits/random.tcc: param_type::_M_initialize and
// operator()): fewer than two weights give the one-outcome distribution, which
// returns 0 without touching the generator; otherwise sum = accumulate(w, 0.0),
// p_i = w_i / sum, cp = partial_sum(p) with its last entry set to 1.0, one
// generate_canonical<double, 53> draw u, and the index of the first cp_i >= u
// (lower_bound).  discrete_draw does the same divisions and additions in the
// same order, so every partial sum is bit-identical, and scans them until the
// first one >= u (the same index: the sequence is non-decreasing and its last
// entry, 1.0, is >= u < 1).  The caller passes sum = accumulate(w, 0.0), which
// the walk needs anyway.  Checked against std::discrete_distribution by
// tests/test_sample_cpu.py.
#ifndef PSX_SAMPLE_H
#define PSX_SAMPLE_H

#include <cstddef>
#include <limits>
#include <random>

namespace psx {

template <class G>
inline size_t discrete_draw(const double* w, size_t n, double sum, G& gen) {
    if (n < 2) return 0;
    const double u = std::generate_canonical<double, std::numeric_limits<double>::digits>(gen);
    double cp = w[0] / sum;
    if (!(cp < u)) return 0;
    for (size_t i = 1; i + 1 < n; i++) {
        cp = cp + w[i] / sum;
        if (!(cp < u)) return i;
    }
    return n - 1;
}

}  // namespace psx

#endif
