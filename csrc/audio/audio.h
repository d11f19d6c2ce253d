// Audio helpers for the desktop-audio path: G.711 mu-law (the WebRTC
// PCMU codec every browser supports; no Opus library exists in this image) and a
// stateful polyphase FIR decimator (48 kHz stereo capture -> 8 kHz mono for PCMU).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mx {
namespace audio {

uint8_t linear_to_ulaw(int16_t pcm);
int16_t ulaw_to_linear(uint8_t u);
std::string encode_ulaw(const int16_t* pcm, size_t n);

// Downmix interleaved `channels`-channel s16 to mono and decimate by an integer factor
// with a windowed-sinc low-pass (Blackman), keeping filter history across calls.
class Decimator {
   public:
    Decimator(int factor, int channels, int taps_per_phase = 16);
    std::vector<int16_t> process(const int16_t* interleaved, size_t frames);
    int factor() const { return factor_; }
    int channels() const { return channels_; }
    const std::vector<float>& taps() const { return h_; }

   private:
    int factor_, channels_;
    std::vector<float> h_;
    std::vector<float> hist_;  // last (taps-1) mono input samples
    int phase_ = 0;            // input samples to skip before the next output
};

}  // namespace audio
}  // namespace mx
