// HPC_Sparse_Matrix.hpp -- the reference's matrix handle, field for field.
//
// Drop-in seam (3) of SURVEY.md section 8(b): a caller built against the
// reference keeps producing this struct (generate_matrix / read_HPC_row) and
// hands it to HPCCG(). Field order and types match the reference declaration
// (HPC_Sparse_Matrix.hpp:54-85 in Dart120/HPCCG-SYCL), including the optional
// MPI block, so objects are layout-compatible with a reference build compiled
// with or without -DUSING_MPI.
//
// The MI355X library reads only the fields that precede the MPI block
// (start_row ... ptr_to_diags), so it accepts either layout.
#ifndef HPCCG_AMD_HPC_SPARSE_MATRIX_HPP
#define HPCCG_AMD_HPC_SPARSE_MATRIX_HPP

// Upper bounds the reference's MPI setup uses (its make_local_matrix aborts
// past them). The MI355X path does not inherit them.
const int max_external = 100000;
const int max_num_messages = 500;
const int max_num_neighbors = max_num_messages;

struct HPC_Sparse_Matrix_STRUCT {
    char* title;
    int start_row;        // first global row owned by this rank
    int stop_row;         // last global row owned by this rank
    int total_nrow;       // global rows over all ranks
    long long total_nnz;  // as stored by the generator (27 * total_nrow, approximate)
    int local_nrow;
    int local_ncol;
    int local_nnz;
    int* nnz_in_row;              // entries per row
    double** ptr_to_vals_in_row;  // row i values start here
    int** ptr_to_inds_in_row;     // row i column indices start here
    double** ptr_to_diags;        // pointer to the diagonal entry of row i
#ifdef USING_MPI
    int num_external;
    int num_send_neighbors;
    int* external_index;
    int* external_local_index;
    int total_to_be_sent;
    int* elements_to_send;
    int* neighbors;
    int* recv_length;
    int* send_length;
    double* send_buffer;
#endif
    double* list_of_vals;  // backing store of all values (owned)
    int* list_of_inds;     // backing store of all indices (owned)
};
typedef struct HPC_Sparse_Matrix_STRUCT HPC_Sparse_Matrix;

#ifdef __cplusplus
// Frees a matrix produced by generate_matrix() of this package.
void destroyMatrix(HPC_Sparse_Matrix*& A);
#endif

#endif
