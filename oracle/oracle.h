/* sputnik-amd ORACLE (test infrastructure only; see oracle.c header). */
#ifndef SPUTNIK_AMD_ORACLE_H_
#define SPUTNIK_AMD_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int oracle_mask_to_bcsr(int rows, int cols, int nnz, const int64_t *perm,
                        int32_t *offsets, int32_t *indices);
void oracle_row_indices(int block_rows, const int32_t *offsets,
                        int16_t *row_indices);
void oracle_transpose(int block_rows, int block_cols, const int32_t *offsets,
                      const int16_t *indices, int32_t *offsets_t,
                      int16_t *indices_t, int32_t *block_offsets);
void oracle_bitmask(int block_rows, int block_cols, const int32_t *offsets,
                    const int16_t *indices, uint64_t *words_out);
void oracle_bcsr_to_dense(int rows, int cols, int bd, const int32_t *offsets,
                          const int16_t *indices, const float *values,
                          float *out);
void oracle_gemm(int m, int n, int k, const float *a, int ta, const float *b,
                 int tb, const uint8_t *a_mask, const uint8_t *b_mask,
                 const uint8_t *out_mask, float *out, int threads);
void oracle_round(const float *in, float *out, int64_t n, int dtype);
int oracle_openmp_threads(void);

#ifdef __cplusplus
}
#endif

#endif /* SPUTNIK_AMD_ORACLE_H_ */
