// Test double of the Ceres 2.0 plug-in interfaces used by include/pba_ceres.h — written from the documented
// declarations (cost_function.h:64-136, sized_cost_function.h, local_parameterization.h,
// evaluation_callback.h:63-76), so the adapter can be compiled and exercised without building Ceres (which
// needs its CMake-generated config.h).  Only the members the adapter and its test use exist here.
#pragma once

#include <cstdint>
#include <vector>

namespace ceres {

class CostFunction {
 public:
  virtual ~CostFunction() {}
  virtual bool Evaluate(double const* const* parameters, double* residuals, double** jacobians) const = 0;
  int num_residuals() const { return num_residuals_; }
  const std::vector<int32_t>& parameter_block_sizes() const { return sizes_; }

 protected:
  void set_num_residuals(int n) { num_residuals_ = n; }
  std::vector<int32_t>* mutable_parameter_block_sizes() { return &sizes_; }

 private:
  int num_residuals_ = 0;
  std::vector<int32_t> sizes_;
};

template <int kNumResiduals, int... Ns>
class SizedCostFunction : public CostFunction {
 public:
  SizedCostFunction() {
    set_num_residuals(kNumResiduals);
    *mutable_parameter_block_sizes() = std::vector<int32_t>{Ns...};
  }
};

class LocalParameterization {
 public:
  virtual ~LocalParameterization() {}
  virtual bool Plus(const double* x, const double* delta, double* x_plus_delta) const = 0;
  virtual bool ComputeJacobian(const double* x, double* jacobian) const = 0;
  virtual int GlobalSize() const = 0;
  virtual int LocalSize() const = 0;
};

class EvaluationCallback {
 public:
  virtual ~EvaluationCallback() {}
  virtual void PrepareForEvaluation(bool evaluate_jacobians, bool new_evaluation_point) = 0;
};

}  // namespace ceres
