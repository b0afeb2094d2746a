# oracle/ceres.mk — TEST-ONLY: the reference's vendored Ceres Solver 2.0.0 compiled from its own sources into
# oracle/_ref/libceres.a, without the reference's CMake.  It follows Ceres' own non-CMake recipe
# (thirdparty/ceres-solver/bazel/ceres.bzl:31-125 source list, :140-200 flags): the EMPTY config header the
# reference ships for such builds (config/ceres/internal/config.h) plus the feature -D defines on the command line,
# Ceres' vendored miniglog for glog, the reference's Eigen 3.3.8.  Nothing is generated and no stand-in is written.
#
# Used only by the checkers: tests/cpp (real-Ceres LM over the GPU EvaluationCallback, include/pba_ceres.h), the
# PhotometricError<8> golden-vector harness and the cpu_baseline.  Outputs go to oracle/_ref/ (git-ignored).
#   make -f ceres.mk -j8        (≈3 min on 8 cores)
REF ?= /root/reference
CERES := $(REF)/thirdparty/ceres-solver
OUT := _ref/ceres
CXX ?= g++

CERES_DEFS := -DCERES_NO_SUITESPARSE -DCERES_NO_CXSPARSE -DCERES_NO_ACCELERATE_SPARSE -DCERES_NO_LAPACK \
              -DCERES_USE_EIGEN_SPARSE -DCERES_USE_CXX_THREADS -DCERES_RESTRICT_SCHUR_SPECIALIZATION \
              -DMAX_LOG_LEVEL=-1
CERES_INC := -I$(CERES)/config -I$(CERES)/include -I$(CERES)/internal -I$(CERES)/internal/ceres/miniglog \
             -I$(REF)/thirdparty/eigen
CERES_FLAGS := -std=c++14 -O2 -DNDEBUG -fPIC -w -pthread $(CERES_DEFS) $(CERES_INC)

# ceres.bzl:31-125 (CERES_SRCS; its split.cc is not in this 2.0.0 tree) + the d_d_d Schur instantiations (restrict_schur_specializations, :149-155)
SRCS := accelerate_sparse array_utils blas block_evaluate_preparer block_jacobian_writer block_jacobi_preconditioner \
  block_random_access_dense_matrix block_random_access_diagonal_matrix block_random_access_matrix \
  block_random_access_sparse_matrix block_sparse_matrix block_structure c_api callbacks canonical_views_clustering \
  cgnr_solver compressed_col_sparse_matrix_utils compressed_row_jacobian_writer compressed_row_sparse_matrix \
  conditioned_cost_function conjugate_gradients_solver context context_impl coordinate_descent_minimizer corrector \
  covariance covariance_impl dense_normal_cholesky_solver dense_qr_solver dense_sparse_matrix detect_structure \
  dogleg_strategy dynamic_compressed_row_jacobian_writer dynamic_compressed_row_sparse_matrix \
  dynamic_sparse_normal_cholesky_solver eigensparse evaluator file function_sample gradient_checker \
  gradient_checking_cost_function gradient_problem gradient_problem_solver is_close implicit_schur_complement \
  inner_product_computer iterative_refiner iterative_schur_complement_solver lapack levenberg_marquardt_strategy \
  line_search line_search_direction line_search_minimizer linear_least_squares_problems linear_operator \
  line_search_preprocessor linear_solver local_parameterization loss_function low_rank_inverse_hessian minimizer \
  normal_prior parallel_for_cxx parallel_for_openmp parallel_utils parameter_block_ordering partitioned_matrix_view \
  polynomial preconditioner preprocessor problem problem_impl program reorder_program residual_block \
  residual_block_utils schur_complement_solver schur_eliminator schur_jacobi_preconditioner schur_templates \
  scratch_evaluate_preparer single_linkage_clustering solver solver_utils sparse_cholesky sparse_matrix \
  sparse_normal_cholesky_solver stringprintf subset_preconditioner suitesparse thread_pool \
  thread_token_provider triplet_sparse_matrix trust_region_minimizer trust_region_preprocessor \
  trust_region_step_evaluator trust_region_strategy types visibility_based_preconditioner visibility wall_time \
  generated/schur_eliminator_d_d_d generated/partitioned_matrix_view_d_d_d miniglog/glog/logging

OBJS := $(addprefix $(OUT)/,$(addsuffix .o,$(SRCS)))

_ref/libceres.a: $(OBJS)
	ar rcs $@ $^

$(OUT)/%.o: $(CERES)/internal/ceres/%.cc
	@mkdir -p $(dir $@)
	$(CXX) $(CERES_FLAGS) -c -o $@ $<

.PHONY: print-flags
print-flags:
	@echo $(CERES_FLAGS)

# ---- real-Ceres drivers over the engine (tests/cpp): linked against _ref/libceres.a and the engine's libpba.so -----
ROOT := ..
PBA_LIB := $(ROOT)/photometric-bundle-adjustment_amd/csrc
DRV_FLAGS := -std=c++17 -O2 -DNDEBUG -w -pthread $(CERES_DEFS) $(CERES_INC) -I$(REF)/thirdparty/Sophus \
             -I$(REF)/include/visnav -I$(ROOT)/include -I$(ROOT)/tests/cpp
DRV_LIBS := _ref/libceres.a -L$(PBA_LIB) -lpba -Wl,-rpath,'$$ORIGIN/../../photometric-bundle-adjustment_amd/csrc' -pthread

drivers: _ref/ceres_lm_driver _ref/adapter_driver _ref/golden_ceres

_ref/ceres_lm_driver: $(ROOT)/tests/cpp/ceres_lm_driver.cpp $(ROOT)/tests/cpp/ceres_functors.h $(ROOT)/include/pba_ceres.h \
                      $(ROOT)/include/pba.h _ref/libceres.a $(PBA_LIB)/libpba.so
	$(CXX) $(DRV_FLAGS) -I$(CERES)/internal/ceres/autodiff_benchmarks -o $@ $< $(DRV_LIBS)

# the adapter driver of tests/test_ceres_adapter.py, against the REAL ceres/ceres.h instead of the test double
_ref/adapter_driver: $(ROOT)/tests/cpp/adapter_driver.cpp $(ROOT)/include/pba_ceres.h $(ROOT)/include/pba.h _ref/libceres.a $(PBA_LIB)/libpba.so
	$(CXX) $(DRV_FLAGS) -o $@ $< $(DRV_LIBS)

# golden vectors from Ceres' own BiCubicInterpolator and PhotometricError<8> (tests/golden/make_ceres_golden.py)
_ref/golden_ceres: golden_ceres.cpp $(ROOT)/tests/cpp/ceres_functors.h _ref/libceres.a
	$(CXX) $(DRV_FLAGS) -I$(CERES)/internal/ceres/autodiff_benchmarks -o $@ $< _ref/libceres.a -pthread

.PHONY: drivers

$(PBA_LIB)/libpba.so: FORCE
	$(MAKE) -s -C $(PBA_LIB) libpba.so

.PHONY: FORCE
FORCE:
