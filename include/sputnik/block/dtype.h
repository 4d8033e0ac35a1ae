// sputnik-amd: element type selector for the extended (bf16-capable) entry
// points. The reference is fp16-only.
#ifndef SPUTNIK_BLOCK_DTYPE_H_
#define SPUTNIK_BLOCK_DTYPE_H_

namespace sputnik {
namespace block {

enum class DataType : int {
  kF16 = 0,   // IEEE binary16 in/out, fp32 accumulate (the reference's type)
  kBF16 = 1,  // bfloat16 in/out, fp32 accumulate
};

}  // namespace block
}  // namespace sputnik

#endif  // SPUTNIK_BLOCK_DTYPE_H_
