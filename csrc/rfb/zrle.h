// Native RFB encoder pieces (replaces x11vnc's LibVNC encoders, reference
// Dockerfile:504-505): ZRLE rectangles (RFC 6143 §7.7.6) with every tile subencoding
// (solid, packed palette 2-16, plain RLE, palette RLE, raw) chosen per 64x64 tile by exact
// output size, over one persistent zlib stream per connection; and the dirty-tile diff of
// two host framebuffers.
#pragma once
#include <zlib.h>

#include <cstdint>
#include <string>
#include <vector>

namespace mx {
namespace rfb {

class ZrleEncoder {
   public:
    explicit ZrleEncoder(int level = 6);
    ~ZrleEncoder();
    ZrleEncoder(const ZrleEncoder&) = delete;
    ZrleEncoder& operator=(const ZrleEncoder&) = delete;

    // One rectangle of a BGRx framebuffer -> "u32 length | zlib bytes" (the ZRLE rectangle
    // body).  perm[k] = source byte (0 B, 1 G, 2 R) of CPIXEL byte k (client pixel format).
    std::string encode(const uint8_t* frame, size_t pitch, int x, int y, int w, int h, const int perm[3]);
    // Tile-subencoding histogram of everything encoded so far (index = subencoding byte).
    const std::vector<uint64_t>& stats() const { return stats_; }

   private:
    void encode_tile(const uint8_t* frame, size_t pitch, int x, int y, int w, int h, const int perm[3]);
    z_stream zs_{};
    std::string raw_;
    std::vector<uint32_t> px_;
    std::vector<uint64_t> stats_ = std::vector<uint64_t>(256, 0);
};

// Per-tile change flags (row-major, ceil(w/tile) x ceil(h/tile)) between two BGRx frames.
std::vector<uint8_t> tile_diff(const uint8_t* cur, const uint8_t* prev, size_t pitch, int w, int h, int tile);

}  // namespace rfb
}  // namespace mx
