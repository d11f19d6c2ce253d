#include "audio.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>

namespace mx {
namespace audio {

// ITU-T G.711 mu-law, 16-bit linear input (bias 0x84, 8 segments, clip at 32635).
uint8_t linear_to_ulaw(int16_t pcm) {
    constexpr int kBias = 0x84, kClip = 32635;
    int v = pcm;
    int mask = 0xFF;
    if (v < 0) {
        v = -v;
        mask = 0x7F;
    }
    v = std::min(v, kClip) + kBias;
    int seg = 0;
    for (int s = v >> 7; s > 1 && seg < 7; s >>= 1) ++seg;
    const int u = (seg << 4) | ((v >> (seg + 3)) & 0x0F);
    return (uint8_t)(u ^ mask);
}

int16_t ulaw_to_linear(uint8_t u) {
    constexpr int kBias = 0x84;
    u = (uint8_t)~u;
    int t = ((u & 0x0F) << 3) + kBias;
    t <<= (u & 0x70) >> 4;
    return (int16_t)((u & 0x80) ? (kBias - t) : (t - kBias));
}

std::string encode_ulaw(const int16_t* pcm, size_t n) {
    std::string out(n, '\0');
    for (size_t i = 0; i < n; ++i) out[i] = (char)linear_to_ulaw(pcm[i]);
    return out;
}

Decimator::Decimator(int factor, int channels, int taps_per_phase) : factor_(factor), channels_(channels) {
    if (factor < 1 || channels < 1 || taps_per_phase < 2) throw std::invalid_argument("bad decimator parameters");
    const int n = factor * taps_per_phase + 1;
    h_.resize(n);
    const double fc = 0.45 / factor;  // cutoff below the new Nyquist
    double sum = 0;
    for (int i = 0; i < n; ++i) {
        const double m = i - (n - 1) / 2.0;
        const double sinc = (m == 0) ? 2 * fc : std::sin(2 * M_PI * fc * m) / (M_PI * m);
        const double w = 0.42 - 0.5 * std::cos(2 * M_PI * i / (n - 1)) + 0.08 * std::cos(4 * M_PI * i / (n - 1));
        h_[i] = (float)(sinc * w);
        sum += h_[i];
    }
    for (auto& x : h_) x = (float)(x / sum);
    hist_.assign(n - 1, 0.f);
}

std::vector<int16_t> Decimator::process(const int16_t* x, size_t frames) {
    const int n = (int)h_.size();
    std::vector<float> buf(hist_);
    buf.reserve(hist_.size() + frames);
    for (size_t f = 0; f < frames; ++f) {
        float s = 0;
        for (int c = 0; c < channels_; ++c) s += x[f * channels_ + c];
        buf.push_back(s / channels_);
    }
    std::vector<int16_t> out;
    out.reserve(frames / factor_ + 1);
    // output k uses inputs buf[i - n + 1 .. i] for i = (n-1) + phase_ + k*factor
    size_t i = (size_t)(n - 1 + phase_);
    for (; i < buf.size(); i += factor_) {
        float acc = 0;
        const float* p = &buf[i - (n - 1)];
        for (int k = 0; k < n; ++k) acc += h_[k] * p[k];
        out.push_back((int16_t)std::lround(std::clamp(acc, -32768.f, 32767.f)));
    }
    phase_ = (int)(i - buf.size());
    hist_.assign(buf.end() - (n - 1), buf.end());
    return out;
}

}  // namespace audio
}  // namespace mx
