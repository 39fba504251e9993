// HPCCG.hpp -- drop-in solver entry with the reference's exact C++ signature
// (HPCCG.hpp:61-63 in Dart120/HPCCG-SYCL). A reference-style main.cpp that
// includes this header and links libhpccg_hip.so runs the CG solve on the
// MI355X instead of the CPU: same arguments, same in/out meaning of x,
// niters, normr and times[] (times[0] total, [1] ddot, [2] waxpby, [3]
// sparsemv, [4] all-reduce, [5] halo exchange; [6] is left to the caller as
// in main.cpp:179-180, plus this library's one-time H2D setup).
#ifndef HPCCG_AMD_HPCCG_HPP
#define HPCCG_AMD_HPCCG_HPP
#include "HPC_Sparse_Matrix.hpp"

int HPCCG(HPC_Sparse_Matrix* A, double* const b, double* const x, const int max_iter,
          const double tolerance, int& niters, double& normr, double* times);

// generate_matrix.hpp:58 (serial / rank 0 of 1, 27-point stencil).
void generate_matrix(int nx, int ny, int nz, HPC_Sparse_Matrix** A, double** x, double** b,
                     double** xexact);
#endif
