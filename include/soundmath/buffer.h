// soundmath/buffer.h -- Buffer<T> (src/buffer.h:9-86): the circular buffer, host side, with the
// reference's unsigned origin / size so the interpolated read keeps its mod-2^32 wrap
// (buffer.h:40-47).  The Delay / Delaybank and Granulator engines keep their own device rings with
// the same indexing (hz_delay.hip, hz_granulator.hip); this class is the host object a demo writes
// (tests/granny.cpp:36-37) and the source a Granulator reads.
#pragma once

#include <vector>

#include "includes.h"

namespace soundmath {

template <typename T>
class Buffer {
public:
    Buffer() = default;
    explicit Buffer(unsigned size) { initialize(size); }
    void initialize(unsigned size = 0) {
        size += (size == 0) ? 1 : 0;   // buffer.h:21: no size zero
        size_ = size;
        origin_ = 0;
        data_.assign(size, T(0));
    }
    void tick() { origin_ = (origin_ + 1) % size_; }   // 33-37
    // linear-interpolated read into the past (40-47)
    T operator()(T position = 0) const {
        const int center = (int)position, before = center + 1;
        const T disp = position - center;
        return data_[(origin_ - center + size_) % size_] * (1 - disp) + data_[(origin_ - before + size_) % size_] * disp;
    }
    // linear-interpolated read of a static buffer (50-57)
    T operator[](T position) const {
        const int center = (int)position, after = (int)((center + 1) % size_);
        const T disp = position - center;
        return data_[(center + size_) % size_] * (1 - disp) + data_[(after + size_) % size_] * disp;
    }
    void write(T value) { data_[origin_] = value; }   // 59-62
    void accum(T value) { data_[origin_] += value; }  // 64-67
    unsigned get_size() const { return size_; }       // 75-78
    T current() const { return data_[origin_]; }      // (the sample at the write position)

private:
    std::vector<T> data_;
    unsigned size_ = 1, origin_ = 0;
};

}  // namespace soundmath
