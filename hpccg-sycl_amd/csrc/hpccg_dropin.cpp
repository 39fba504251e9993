// hpccg_dropin.cpp -- C++ entry points with the reference signatures
// (HPCCG.hpp:61-63, generate_matrix.hpp:58) forwarding to the C ABI.
#include <iostream>

#include "../../include/HPCCG.hpp"
#include "../../include/hpccg_hip.h"

int HPCCG(HPC_Sparse_Matrix* A, double* const b, double* const x, const int max_iter,
          const double tolerance, int& niters, double& normr, double* times)
{
    int it = 0;
    double nr = 0.0;
    const int rc = hpccg_hip_HPCCG(A, b, x, max_iter, tolerance, &it, &nr, times);
    if (rc) std::cerr << "hpccg_hip: " << hpccg_hip_last_error() << std::endl;
    niters = it;
    normr = nr;
    return rc;
}

void generate_matrix(int nx, int ny, int nz, HPC_Sparse_Matrix** A, double** x, double** b,
                     double** xexact)
{
    hpccg_generate_matrix(nx, ny, nz, 0, 1, 0, A, x, b, xexact);
}
