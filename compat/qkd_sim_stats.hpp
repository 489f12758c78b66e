// qkd_sim_stats.hpp — the per-QBER-point reduction of QKD_LDPC_batch_simulation
// (reference src/simulation.cpp:252-312), restated with the reference's exact
// double arithmetic and loop order so that the CSV values agree to the last
// printed digit: only trials whose syndrome matched contribute; mean by a
// running double sum; population standard deviation by a second pass; min is
// reported as 0 when it stayed at the iteration cap (:306).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstddef>

namespace qkdsim {

struct PointStats {
    size_t trials_successful_sp = 0;
    size_t trials_successful_ldpc = 0;
    size_t iterations_successful_sp_max = 0;
    size_t iterations_successful_sp_min = 0;
    double iterations_successful_sp_mean = 0;
    double iterations_successful_sp_std_dev = 0;
    double ratio_trials_successful_sp = 0;
    double ratio_trials_successful_ldpc = 0;
};

// trial(k, sp_ok, keys_ok, iterations) fills trial k's outcome.
template <typename Trial>
PointStats reduce_point(size_t trials, size_t max_iterations, Trial trial) {
    PointStats s;
    size_t it_min = max_iterations;
    for (size_t k = 0; k < trials; ++k) {
        bool sp = false, ko = false;
        size_t it = 0;
        trial(k, sp, ko, it);
        if (!sp) continue;
        s.trials_successful_sp++;
        s.iterations_successful_sp_max = std::max(s.iterations_successful_sp_max, it);
        it_min = std::min(it_min, it);
        if (ko) s.trials_successful_ldpc++;
        s.iterations_successful_sp_mean += static_cast<double>(it);
    }
    if (s.trials_successful_sp > 0) {
        s.iterations_successful_sp_mean /= static_cast<double>(s.trials_successful_sp);
        for (size_t k = 0; k < trials; ++k) {
            bool sp = false, ko = false;
            size_t it = 0;
            trial(k, sp, ko, it);
            if (sp) s.iterations_successful_sp_std_dev += std::pow(static_cast<double>(it) - s.iterations_successful_sp_mean, 2);
        }
        s.iterations_successful_sp_std_dev /= static_cast<double>(s.trials_successful_sp);
        s.iterations_successful_sp_std_dev = std::sqrt(s.iterations_successful_sp_std_dev);
    }
    s.iterations_successful_sp_min = (it_min == max_iterations) ? 0 : it_min;
    s.ratio_trials_successful_ldpc = static_cast<double>(s.trials_successful_ldpc) / trials;
    s.ratio_trials_successful_sp = static_cast<double>(s.trials_successful_sp) / trials;
    return s;
}

}  // namespace qkdsim
