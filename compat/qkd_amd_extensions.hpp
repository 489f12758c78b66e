// qkd_amd_extensions.hpp — batched entry points the compatibility shim adds
// on top of the reference API (no reference counterpart: the reference runs
// one trial per thread-pool task, simulation.cpp:244-249).
#pragma once
#include <cstddef>
#include <vector>

#include "qkd_reference_api.hpp"

// run_trial (simulation.cpp:161-189) for seeds[k] + seed_offset, k < count, as
// device batches; element k equals run_trial(matrix, QBER, seeds[k] + seed_offset).
// Throws std::runtime_error("Key size '<N>' is too small for QBER.") like run_trial.
std::vector<trial_result> qkd_amd_run_trials(const H_matrix &matrix, double QBER, const size_t *seeds,
                                             size_t count, size_t seed_offset);

// The shim's device (default 0) and decoder variant for every later call:
// "sp_f64" (default: the reference's decoder bit for bit), "sp_f32",
// "minsum" or "minsum_sc" (QKD_VARIANT_* of include/qkd_ldpc.h). The
// reference's only decoder switch is the clamp (CFG), so these are the
// shim's own settings; no environment variable is read. An unknown name
// throws std::runtime_error("... unknown decoder variant '<name>'").
void qkd_amd_set_device(int device);
void qkd_amd_set_variant(const char *name);
