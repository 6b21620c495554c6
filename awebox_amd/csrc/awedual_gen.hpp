// Internal interface between awedual.hip (the handle and the C ABI) and awedual_gen.hip (the
// generated instance-minor evaluation path of the dual-kite NLP).  Not part of include/awedual.h.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "dual_tables.hpp"

namespace dgen {

struct Plan;   // device tables and scratch of the generated path for one handle

// Builds the plan for tables T, the model constants and the batch.  Returns AWE_OK with *out = nullptr
// and `why` set when the generated code does not serve these constants (other tether element count or
// stability-derivative structure); an error code and `err` on a HIP failure.
int create(const dlt::Tables& T, const std::vector<double>& consts, int batch, Plan** out, std::string& why,
           std::string& err);
void destroy(Plan* p);

// f [B], g [B][n_g] (per instance), grad_f and J_g instance-minor (grad_f[i * ldj + b],
// jac[e * ldj + b]); cst: the model constants on the device
int eval(Plan* p, const double* cst, const double* V, const double* P, double* f, double* g, double* grad_f,
         double* jac, size_t ldj, hipStream_t s, std::string& err);

// HIP-event times of the last eval: input transposition, node kernel, interval kernel, finalize (ms)
int last_ms(Plan* p, float ms[4], std::string& err);

}  // namespace dgen
