// qkd_reference_api.hpp — the reference's hot-path C++ interface, as the
// compatibility shim (qkd_ldpc_algorithm_amd.cpp) needs it.
//
// This header exists for building and testing the shim OUTSIDE the reference
// tree. Inside ColdCloudd/QKD_LDPC a maintainer replaces it by a forwarder to
// the reference's own headers:
//     #include "qkd_ldpc_algorithm.hpp"
//     #include "simulation.hpp"
// so the shim then compiles against the real declarations. Every type and
// prototype below states the reference declaration it mirrors; field names,
// types and order match them (H_matrix and the result structs cross between
// the reference's code and the shim by reference).
#pragma once
#include <cstddef>
#include <filesystem>
#include <string>
#include <vector>

namespace fs = std::filesystem;

// src/array_and_matrix_operations.hpp:16-27
struct H_matrix
{
    int **bit_nodes = nullptr;
    int *bit_nodes_weight = nullptr;
    int **check_nodes = nullptr;
    int *check_nodes_weight = nullptr;
    size_t num_bit_nodes{};
    size_t num_check_nodes{};
    size_t max_bit_nodes_weight{};
    size_t max_check_nodes_weight{};
    bool is_regular{};
};

// src/qkd_ldpc_algorithm.hpp:14-24
struct SP_result
{
    size_t iterations_num{};
    bool syndromes_match{};
};

struct LDPC_result
{
    SP_result sp_res{};
    bool keys_match{};
};

// src/config.hpp:14-21, :23-63 (the fields the hot path and the batch driver read)
struct R_QBER_params
{
    double code_rate{};
    double QBER_begin{};
    double QBER_end{};
    double QBER_step{};
};

struct config_data
{
    size_t THREADS_NUMBER{};
    size_t TRIALS_NUMBER{};
    size_t SIMULATION_SEED{};
    bool INTERACTIVE_MODE{};
    size_t SUM_PRODUCT_MAX_ITERATIONS{};
    bool USE_DENSE_MATRICES{};
    bool TRACE_QKD_LDPC{};
    bool TRACE_SUM_PRODUCT{};
    bool TRACE_SUM_PRODUCT_LLR{};
    bool ENABLE_SUM_PRODUCT_MSG_LLR_THRESHOLD{};
    double SUM_PRODUCT_MSG_LLR_THRESHOLD{};
    std::vector<R_QBER_params> R_QBER_PARAMETERS{};
};

// src/config.hpp:65 (defined by the reference's main.cpp:13; by the test driver here)
extern config_data CFG;

// src/simulation.hpp:16-43
struct sim_input
{
    fs::path matrix_path{};
    std::vector<double> QBER{};
    H_matrix matrix{};
};

struct trial_result
{
    LDPC_result ldpc_res{};
    double initial_QBER{};
};

struct sim_result
{
    size_t sim_number{};
    std::string matrix_filename{};
    bool is_regular{};
    size_t num_bit_nodes{};
    size_t num_check_nodes{};
    double initial_QBER{};
    size_t iterations_successful_sp_max{};
    size_t iterations_successful_sp_min{};
    double iterations_successful_sp_mean{};
    double iterations_successful_sp_std_dev{};
    double ratio_trials_successful_sp{};
    double ratio_trials_successful_ldpc{};
};

// src/qkd_ldpc_algorithm.hpp:26-31
SP_result sum_product_decoding_regular(const double *const bit_array_llr, const H_matrix &matrix, const int *const syndrome,
                                       const size_t &max_num_iterations, const double &msg_threshold, int *const bit_array_out);
SP_result sum_product_decoding_irregular(const double *const bit_array_llr, const H_matrix &matrix, const int *const syndrome,
                                         const size_t &max_num_iterations, const double &msg_threshold, int *const bit_array_out);
LDPC_result QKD_LDPC_regular(const int *const alice_bit_array, const int *const bob_bit_array, const double &QBER, const H_matrix &matrix);
LDPC_result QKD_LDPC_irregular(const int *const alice_bit_array, const int *const bob_bit_array, const double &QBER, const H_matrix &matrix);

// src/array_and_matrix_operations.hpp:39-40
void calculate_syndrome_regular(const int *const bit_array, const H_matrix &matrix, int *const syndrome_out);
void calculate_syndrome_irregular(const int *const bit_array, const H_matrix &matrix, int *const syndrome_out);

// src/simulation.hpp:49-50
trial_result run_trial(const H_matrix &matrix, const double QBER, size_t seed);
std::vector<sim_result> QKD_LDPC_batch_simulation(const std::vector<sim_input> &sim_in);
