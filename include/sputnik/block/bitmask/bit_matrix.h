// sputnik-amd: host view of the block bit matrix (reference
// sputnik/block/bitmask/bit_matrix.h:10-60). Rows of ceil(columns / 64)
// uint64 words; bit j % 64 of word j / 64 of row i marks block (i, j). Only
// the layout and its size matter to callers: the device builder is Bitmask().
#ifndef SPUTNIK_BLOCK_BITMASK_BIT_MATRIX_H_
#define SPUTNIK_BLOCK_BITMASK_BIT_MATRIX_H_

#include <cstddef>
#include <cstdint>
#include <vector>

namespace sputnik {
namespace block {

class BitMatrix {
 public:
  static constexpr int kAlignment = 64;  // bits per word

  static size_t WordsPerRow(int columns) {
    return static_cast<size_t>((columns + kAlignment - 1) / kAlignment);
  }
  static size_t SizeInBytes(int rows, int columns) {
    return WordsPerRow(columns) * static_cast<size_t>(rows) *
           sizeof(uint64_t);
  }

  BitMatrix(int rows, int columns)
      : rows_(rows),
        words_per_row_(WordsPerRow(columns)),
        data_(words_per_row_ * static_cast<size_t>(rows), 0) {}

  bool Get(int i, int j) const {
    return (data_[i * words_per_row_ + j / kAlignment] >> (j % kAlignment)) &
           1ull;
  }
  void Set(int i, int j) {
    data_[i * words_per_row_ + j / kAlignment] |= 1ull << (j % kAlignment);
  }
  uint64_t *Data() { return data_.data(); }
  const uint64_t *Data() const { return data_.data(); }
  size_t Bytes() const { return data_.size() * sizeof(uint64_t); }
  int Rows() const { return rows_; }

 private:
  int rows_;
  size_t words_per_row_;
  std::vector<uint64_t> data_;
};

}  // namespace block
}  // namespace sputnik

#endif  // SPUTNIK_BLOCK_BITMASK_BIT_MATRIX_H_
