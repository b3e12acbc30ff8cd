// soundmath/audio.h -- a file-backed stand-in for the reference's PortAudio engine
// (src/audio.h:11-151), so instruments written against it run headless.
//
// The reference opens a duplex PortAudio stream at SR with `bsize` frames per buffer and calls
// process(const float* in, float* out) per buffer with interleaved float32 channels.  Here
// startup(in, out) runs that same callback over a WAV file (or silence) instead of a sound
// card, synchronously, and writes the output to a WAV file:
//     Audio A(process, BSIZE);                  // unchanged demo code
//     Audio::offline("in.wav", "out.wav");      // before startup (or HZ_AUDIO_IN / HZ_AUDIO_OUT)
//     A.startup(1, 1, true);                    // runs the whole input, then returns
//     A.shutdown();
// Input WAV: PCM 16/24/32-bit or IEEE float32/64, any channel count (channels are mapped to
// the `in` channels requested: extra ones dropped, missing ones zero; a mono file feeds every
// input channel).  Without an input file, HZ_AUDIO_SECONDS (default 1) of silence is fed.
// Output: IEEE float32 WAV with `out` channels at SR.  finished() turns true after startup()
// so demo loops (`while (running) Pa_Sleep(5)`) can stop.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "hz.h"

namespace soundmath {

const int def_bsize = 16;

namespace wav {

struct Data {
    int channels = 0, rate = 0;
    std::vector<float> samples;   // interleaved
};

inline uint32_t rd32(const unsigned char* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
inline uint16_t rd16(const unsigned char* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

inline Data read(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("wav::read: cannot open " + path);
    std::vector<unsigned char> b;
    unsigned char chunk[65536];
    size_t got;
    while ((got = std::fread(chunk, 1, sizeof(chunk), f)) > 0) b.insert(b.end(), chunk, chunk + got);
    std::fclose(f);
    if (b.size() < 12 || std::memcmp(b.data(), "RIFF", 4) || std::memcmp(b.data() + 8, "WAVE", 4))
        throw std::runtime_error("wav::read: not a RIFF/WAVE file: " + path);
    Data d;
    int fmt = 0, bits = 0;
    size_t pos = 12;
    while (pos + 8 <= b.size()) {
        const uint32_t len = rd32(&b[pos + 4]);
        const unsigned char* body = &b[pos + 8];
        if (pos + 8 + len > b.size()) throw std::runtime_error("wav::read: truncated chunk in " + path);
        if (!std::memcmp(&b[pos], "fmt ", 4)) {
            fmt = rd16(body);
            d.channels = rd16(body + 2);
            d.rate = (int)rd32(body + 4);
            bits = rd16(body + 14);
            if (fmt == 0xFFFE && len >= 26) fmt = rd16(body + 24);   // WAVE_FORMAT_EXTENSIBLE subformat
        } else if (!std::memcmp(&b[pos], "data", 4)) {
            if (!d.channels || !bits) throw std::runtime_error("wav::read: data before fmt in " + path);
            const size_t width = bits / 8, count = len / width;
            d.samples.resize(count);
            for (size_t i = 0; i < count; ++i) {
                const unsigned char* s = body + i * width;
                if (fmt == 3 && bits == 32) {
                    float v;
                    std::memcpy(&v, s, 4);
                    d.samples[i] = v;
                } else if (fmt == 3 && bits == 64) {
                    double v;
                    std::memcpy(&v, s, 8);
                    d.samples[i] = (float)v;
                } else if (fmt == 1 && bits == 16) {
                    d.samples[i] = (int16_t)rd16(s) / 32768.0f;
                } else if (fmt == 1 && bits == 24) {
                    int32_t v = s[0] | (s[1] << 8) | (s[2] << 16);
                    if (v & 0x800000) v -= 0x1000000;
                    d.samples[i] = v / 8388608.0f;
                } else if (fmt == 1 && bits == 32) {
                    d.samples[i] = (float)((int32_t)rd32(s) / 2147483648.0);
                } else {
                    throw std::runtime_error("wav::read: unsupported format in " + path);
                }
            }
        }
        pos += 8 + len + (len & 1);
    }
    if (!d.channels) throw std::runtime_error("wav::read: no fmt chunk in " + path);
    return d;
}

inline void write(const std::string& path, const float* samples, size_t frames, int channels, int rate) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("wav::write: cannot open " + path);
    auto w32 = [&](uint32_t v) {
        unsigned char c[4] = {(unsigned char)v, (unsigned char)(v >> 8), (unsigned char)(v >> 16), (unsigned char)(v >> 24)};
        std::fwrite(c, 1, 4, f);
    };
    auto w16 = [&](uint16_t v) {
        unsigned char c[2] = {(unsigned char)v, (unsigned char)(v >> 8)};
        std::fwrite(c, 1, 2, f);
    };
    const uint32_t bytes = (uint32_t)(frames * channels * 4);
    std::fwrite("RIFF", 1, 4, f);
    w32(36 + bytes);
    std::fwrite("WAVEfmt ", 1, 8, f);
    w32(16);
    w16(3);   // IEEE float
    w16((uint16_t)channels);
    w32((uint32_t)rate);
    w32((uint32_t)(rate * channels * 4));
    w16((uint16_t)(channels * 4));
    w16(32);
    std::fwrite("data", 1, 4, f);
    w32(bytes);
    std::fwrite(samples, 4, frames * channels, f);
    std::fclose(f);
}

}  // namespace wav

class Audio {
public:
    int bsize;
    int (*process)(const float*, float*);

    Audio(int (*processor)(const float* in, float* out), int bsize = def_bsize) : bsize(bsize), process(processor) {}

    // where startup() reads and writes (empty input: silence)
    static void offline(const std::string& in_wav, const std::string& out_wav) {
        paths().in = in_wav;
        paths().out = out_wav;
    }
    static void initialize(bool report = false, int* def_in = nullptr, int* def_out = nullptr) {
        if (report) std::cout << "offline audio (files, no device)\n";
        if (def_in) *def_in = 0;
        if (def_out) *def_out = 0;
    }

    // src/audio.h:76-129: opens the stream and starts the callbacks; here the callbacks run
    // over the whole input before returning
    void startup(int in = 1, int out = 2, bool report = true, int in_device_id = -1, int out_device_id = -1) {
        (void)in_device_id;
        (void)out_device_id;
        std::string in_path = paths().in, out_path = paths().out;
        if (in_path.empty() && std::getenv("HZ_AUDIO_IN")) in_path = std::getenv("HZ_AUDIO_IN");
        if (out_path.empty() && std::getenv("HZ_AUDIO_OUT")) out_path = std::getenv("HZ_AUDIO_OUT");
        if (out_path.empty()) out_path = "out.wav";
        wav::Data src;
        size_t frames;
        if (!in_path.empty()) {
            src = wav::read(in_path);
            if (src.rate != SR && report)
                std::cout << "warning: " << in_path << " is " << src.rate << " Hz, processed as " << SR << " Hz\n";
            frames = src.samples.size() / src.channels;
        } else {
            const char* sec = std::getenv("HZ_AUDIO_SECONDS");
            frames = (size_t)((sec ? std::atof(sec) : 1.0) * SR);
        }
        const size_t blocks = (frames + bsize - 1) / bsize;
        std::vector<float> ib((size_t)bsize * in), ob((size_t)bsize * out), result(blocks * bsize * out);
        for (size_t blk = 0; blk < blocks; ++blk) {
            for (int i = 0; i < bsize; ++i) {
                const size_t t = blk * bsize + i;
                for (int c = 0; c < in; ++c) {
                    float v = 0.f;
                    if (t < frames && src.channels)
                        v = src.channels == 1 ? src.samples[t] : (c < src.channels ? src.samples[t * src.channels + c] : 0.f);
                    ib[(size_t)i * in + c] = v;
                }
            }
            std::fill(ob.begin(), ob.end(), 0.f);
            process(ib.data(), ob.data());   // src/audio.h:139-148
            std::memcpy(&result[blk * bsize * out], ob.data(), sizeof(float) * ob.size());
        }
        wav::write(out_path, result.data(), frames, out, SR);
        if (report)
            std::cout << "offline audio: " << frames << " frames x " << in << " in -> " << out << " out, " << out_path
                      << "\n";
        done_ = true;
    }
    void shutdown() {}
    bool finished() const { return done_; }

private:
    struct Paths {
        std::string in, out;
    };
    static Paths& paths() {
        static Paths p;
        return p;
    }
    bool done_ = false;
};

}  // namespace soundmath
