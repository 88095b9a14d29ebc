// Internal (non-ABI) reduction helpers shared by the kernel files.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tvq {
// out[j] (+)= sum_{p<P} in[p*ld + j]; L > 0: split output rows of length L into
// out (first L-1 columns, dense) and out2 (last column).  scratch: reduce_rows_scratch floats.
int64_t reduce_rows_scratch(int64_t P, int64_t N);
void reduce_rows(const float* in, int64_t P, int64_t N, int64_t ld, float* out, float* out2,
                 int64_t L, int accumulate, float* scratch, hipStream_t st);
// Batched single-level reduce_rows (P <= RR_ONE = 256 rows, ld = N): each job gives the
// result of the matching reduce_rows call bit for bit, for many slabs in one launch.
struct RrJob {
  const float* in;
  float* out;
  float* out2;
  int64_t P, N, L;
  int accumulate;
};
constexpr int RR_ONE_ROWS = 256;
void reduce_rows_batch(const RrJob* jobs, int n, hipStream_t st);
// stable group-by of indices in [0,V): offsets[V+1], perm[M]; scratch: group_by_scratch_ints ints
int64_t group_by_scratch_ints(int64_t M, int64_t V);
// counts / countsf (optional, V each): the per-value counts as int32 and float
void group_by_i32(const int32_t* idx, int64_t M, int64_t V, int* offsets, int* perm, int* scratch,
                  hipStream_t st, int32_t* counts = nullptr, float* countsf = nullptr);
void group_by_i64(const int64_t* idx, int64_t M, int64_t V, int* offsets, int* perm, int* scratch,
                  hipStream_t st);
// Rows for seg_rowsum: row m -> src + (m / N)*sB + (m % N)*sN, element d at + d*sD.
// Optional dropout mask (nn.Embedding backward of the token-embedding dropout):
// element (m, d) kept iff uniform01(mix_seed(seed_ptr, offset), m*D + d) >= drop_p,
// unless the row's value equals mask_id.
struct SegRows {
  const float* src;
  int64_t N, sB, sN, sD;
  int D;  // <= 512
  float drop_p;
  const int64_t* seed_ptr;
  uint64_t offset;
  int64_t mask_id;
};
// out[v, :] (+)= sum of rows of value v (perm order); part: seg_rowsum_scratch_floats floats;
// seg_start: group_by_seg_start(scratch) of the same group_by call.
int64_t seg_rowsum_scratch_floats(int64_t M, int64_t V, int64_t D);
int* group_by_seg_start(int* scratch, int64_t M, int64_t V);
void seg_rowsum(const SegRows& s, const int* offsets, const int* perm, const int* seg_start,
                int64_t M, int64_t V, float* out, int accumulate, float* part, hipStream_t st);
// the mean of a masked cross-entropy from per-block (loss sum, count) pairs part[2 P]:
// out = {sum / count, count} (tvq_xf.hip masked_ce_final_kernel), one block
void masked_ce_final(const float* part, int P, float* out, hipStream_t st);
}  // namespace tvq
