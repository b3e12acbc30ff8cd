// hz_chain.h -- a generator bank's block feeding a Delaybank in one launch (hz_bowl.hip
// hz_bowl_fill_delaybank): the Delaybank side of the hand-off.  The reference's pattern
// `bowl.fill(buf, 1024); bank.process(buf, out, 1024);` is two objects and, on
// the GPU, four launches per block; when every live tap of the bank reads either the current sample
// (age 0) or a sample at least one block old that is not overwritten within the block (age in
// [n, size - n]), each sample of the block is independent of the block's other samples, so a
// workgroup can produce its samples' generator output and then every line of the bank for them.
#pragma once

#include "hz_common.h"

struct hz_dly;

namespace hz_chain {

constexpr int kMaxTaps = 8;       // taps per line (forward and feedback each) the fused kernel holds

struct DlyBlock {
    const int4* taps;     // [N][2S] {thr, age_nowrap, age_wrap, 0}
    const float* gains;   // [N][2S]
    float* rx;            // [N][size] input rings
    float* ry;            // [N][size] output rings
    unsigned size, o0;
    int N, S;
    hipStream_t stream;
};

// the float bank's block arguments for a call of n samples; *fusable: every live tap age is 0 or
// in [n, size - n] (and 2 n <= size, S <= kMaxTaps): the block may run inside another kernel
int dly_block_begin(hz_dly* h, long n, DlyBlock* b, bool* fusable);
// after such a launch: the origin moves n samples, block work pending on the bank's stream
void dly_block_end(hz_dly* h, long n);

}  // namespace hz_chain
