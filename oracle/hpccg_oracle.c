/*
 * hpccg_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference HPCCG hot path (Dart120/HPCCG-SYCL), used
 * as the parity checker for the HIP path and as the `cpu_baseline` ("port")
 * leg of bench.py. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline may load this library; the product path (hpccg-sycl_amd/)
 * never links or calls it.
 *
 * Pinning: tests/test_oracle.py checks this file against golden vectors
 * produced by the reference itself, compiled from its own sources into
 * oracle/_ref/ (oracle/Makefile, tests/golden/make_golden.py), and against the
 * reference's own sample output /root/reference/out.txt (copied as data into
 * tests/golden/out_10x10x10_150.txt). With nthreads == 1 every function is
 * bitwise identical to the reference serial build (same loop orders, no FMA
 * contraction: compile with -ffp-contract=off).
 *
 * Matrix layout here is plain CSR with 64-bit row pointers (the reference
 * keeps pointer-per-row CSR, HPC_Sparse_Matrix.hpp:54-85; entry order per
 * row is preserved, which is all that matters for rounding).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static double oracle_now(void)
{
    struct timeval tp;
    gettimeofday(&tp, NULL);
    return (double)tp.tv_sec + (double)tp.tv_usec * 1e-6;
}

/* Number of stored entries the generator produces for one rank's slab.
 * Follows generate_matrix.cpp:251-281 (same acceptance test). */
long long oracle_count_nnz(int nx, int ny, int nz, int rank, int size, int use_7pt)
{
    long long local_nrow = (long long)nx * ny * nz;
    long long total_nrow = local_nrow * size;
    long long start_row = local_nrow * rank;
    long long nnz = 0;
    for (int iz = 0; iz < nz; iz++)
        for (int iy = 0; iy < ny; iy++)
            for (int ix = 0; ix < nx; ix++) {
                long long currow = start_row + (long long)iz * nx * ny + (long long)iy * nx + ix;
                for (int sz = -1; sz <= 1; sz++)
                    for (int sy = -1; sy <= 1; sy++)
                        for (int sx = -1; sx <= 1; sx++) {
                            long long curcol = currow + (long long)sz * nx * ny + (long long)sy * nx + sx;
                            if (ix + sx >= 0 && ix + sx < nx && iy + sy >= 0 && iy + sy < ny &&
                                curcol >= 0 && curcol < total_nrow &&
                                (!use_7pt || sz * sz + sy * sy + sx * sx <= 1))
                                nnz++;
                        }
            }
    return nnz;
}

/* generate_matrix.cpp:196-307: 27-pt (or 7-pt) stencil on a z-stacked chimney,
 * global column indices, diagonal 27.0, off-diagonal -1.0, x0 = 0,
 * b = 27 - (nnz_row - 1), xexact = 1. Caller allocates row_ptr[nrow+1],
 * cols/vals[oracle_count_nnz(...)], x/b/xexact[nrow]. */
int oracle_generate(int nx, int ny, int nz, int rank, int size, int use_7pt,
                    long long *row_ptr, int *cols, double *vals,
                    double *x, double *b, double *xexact)
{
    long long local_nrow = (long long)nx * ny * nz;
    long long total_nrow = local_nrow * size;
    long long start_row = local_nrow * rank;
    long long k = 0;
    row_ptr[0] = 0;
    for (int iz = 0; iz < nz; iz++)
        for (int iy = 0; iy < ny; iy++)
            for (int ix = 0; ix < nx; ix++) {
                long long lrow = (long long)iz * nx * ny + (long long)iy * nx + ix;
                long long currow = start_row + lrow;
                int nnzrow = 0;
                for (int sz = -1; sz <= 1; sz++)
                    for (int sy = -1; sy <= 1; sy++)
                        for (int sx = -1; sx <= 1; sx++) {
                            long long curcol = currow + (long long)sz * nx * ny + (long long)sy * nx + sx;
                            if (ix + sx >= 0 && ix + sx < nx && iy + sy >= 0 && iy + sy < ny &&
                                curcol >= 0 && curcol < total_nrow &&
                                (!use_7pt || sz * sz + sy * sy + sx * sx <= 1)) {
                                vals[k] = (curcol == currow) ? 27.0 : -1.0;
                                cols[k] = (int)curcol;
                                k++;
                                nnzrow++;
                            }
                        }
                row_ptr[lrow + 1] = k;
                x[lrow] = 0.0;
                b[lrow] = 27.0 - ((double)(nnzrow - 1));
                xexact[lrow] = 1.0;
            }
    return 0;
}

/* HPC_sparsemv.cpp:68-89: y[i] = sum_j vals[j]*x[cols[j]] in entry order. */
void oracle_sparsemv(int nrow, const long long *row_ptr, const int *cols, const double *vals,
                     const double *x, double *y, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads) if (nthreads > 1)
#endif
    for (int i = 0; i < nrow; i++) {
        double sum = 0.0;
        for (long long j = row_ptr[i]; j < row_ptr[i + 1]; j++)
            sum += vals[j] * x[cols[j]];
        y[i] = sum;
    }
    (void)nthreads;
}

/* ddot.cpp:60-88 (x == y special case computes the same products). */
double oracle_ddot(int n, const double *x, const double *y, int nthreads)
{
    double local_result = 0.0;
    if (nthreads <= 1) {
        for (int i = 0; i < n; i++) local_result += x[i] * y[i];
        return local_result;
    }
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads) reduction(+ : local_result)
#endif
    for (int i = 0; i < n; i++) local_result += x[i] * y[i];
    return local_result;
}

/* waxpby.cpp:69-93: the reference's three branches. alpha==1 / beta==1 only
 * drop an exact multiply by 1.0, so all branches round like the general form. */
void oracle_waxpby(int n, double alpha, const double *x, double beta, const double *y,
                   double *w, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (alpha == 1.0) {
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads) if (nthreads > 1)
#endif
        for (int i = 0; i < n; i++) w[i] = x[i] + beta * y[i];
    } else if (beta == 1.0) {
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads) if (nthreads > 1)
#endif
        for (int i = 0; i < n; i++) w[i] = alpha * x[i] + y[i];
    } else {
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads) if (nthreads > 1)
#endif
        for (int i = 0; i < n; i++) w[i] = alpha * x[i] + beta * y[i];
    }
    (void)nthreads;
}

/* HPCCG.cpp:312-402 (serial / OpenMP path, no MPI). Extra output: when
 * normr_trace != NULL, normr_trace[k] receives the normr value computed in
 * iteration k (k >= 1), normr_trace[0] the initial residual; entries past
 * niters are left untouched. times[0..4] as in the reference. */
int oracle_hpccg(int nrow, const long long *row_ptr, const int *cols, const double *vals,
                 const double *b, double *x, int max_iter, double tolerance,
                 int *niters_out, double *normr_out, double *times, double *normr_trace,
                 int nthreads)
{
    double t_begin = oracle_now();
    double t0 = 0.0, t1 = 0.0, t2 = 0.0, t3 = 0.0, t4 = 0.0;
    int niters = 0;
    double *r = (double *)malloc(sizeof(double) * (size_t)(nrow > 0 ? nrow : 1));
    double *p = (double *)malloc(sizeof(double) * (size_t)(nrow > 0 ? nrow : 1));
    double *Ap = (double *)malloc(sizeof(double) * (size_t)(nrow > 0 ? nrow : 1));
    double normr = 0.0, rtrans = 0.0, oldrtrans = 0.0;
#define TICK() t0 = oracle_now()
#define TOCK(t) t += oracle_now() - t0
    TICK(); oracle_waxpby(nrow, 1.0, x, 0.0, x, p, nthreads); TOCK(t2);
    TICK(); oracle_sparsemv(nrow, row_ptr, cols, vals, p, Ap, nthreads); TOCK(t3);
    TICK(); oracle_waxpby(nrow, 1.0, b, -1.0, Ap, r, nthreads); TOCK(t2);
    TICK(); rtrans = oracle_ddot(nrow, r, r, nthreads); TOCK(t1);
    normr = sqrt(rtrans);
    if (normr_trace) normr_trace[0] = normr;
    for (int k = 1; k < max_iter && normr > tolerance; k++) {
        if (k == 1) {
            TICK(); oracle_waxpby(nrow, 1.0, r, 0.0, r, p, nthreads); TOCK(t2);
        } else {
            oldrtrans = rtrans;
            TICK(); rtrans = oracle_ddot(nrow, r, r, nthreads); TOCK(t1);
            double beta = rtrans / oldrtrans;
            TICK(); oracle_waxpby(nrow, 1.0, r, beta, p, p, nthreads); TOCK(t2);
        }
        normr = sqrt(rtrans);
        if (normr_trace) normr_trace[k] = normr;
        TICK(); oracle_sparsemv(nrow, row_ptr, cols, vals, p, Ap, nthreads); TOCK(t3);
        double alpha;
        TICK(); alpha = oracle_ddot(nrow, p, Ap, nthreads); TOCK(t1);
        alpha = rtrans / alpha;
        TICK(); oracle_waxpby(nrow, 1.0, x, alpha, p, x, nthreads);
        oracle_waxpby(nrow, 1.0, r, -alpha, Ap, r, nthreads); TOCK(t2);
        niters = k;
    }
#undef TICK
#undef TOCK
    if (times) {
        times[1] = t1; times[2] = t2; times[3] = t3; times[4] = t4;
        times[0] = oracle_now() - t_begin;
    }
    *niters_out = niters;
    *normr_out = normr;
    free(r); free(p); free(Ap);
    return 0;
}

/* compute_residual.cpp:59-81: max |v1 - v2|. */
double oracle_compute_residual(int n, const double *v1, const double *v2)
{
    double res = 0.0;
    for (int i = 0; i < n; i++) {
        double d = fabs(v1[i] - v2[i]);
        if (d > res) res = d;
    }
    return res;
}

int oracle_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
