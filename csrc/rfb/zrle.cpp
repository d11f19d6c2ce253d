#include "zrle.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace mx {
namespace rfb {

namespace {
constexpr int kTile = 64;

void put_cpixel(std::string& o, uint32_t v) {
    o.push_back((char)(v & 0xff));
    o.push_back((char)((v >> 8) & 0xff));
    o.push_back((char)((v >> 16) & 0xff));
}

// run length: one or more bytes summing to len-1, all but the last equal to 255
void put_run(std::string& o, int len) {
    int r = len - 1;
    while (r >= 255) {
        o.push_back((char)255);
        r -= 255;
    }
    o.push_back((char)r);
}

int run_bytes(int len) { return (len - 1) / 255 + 1; }
}  // namespace

ZrleEncoder::ZrleEncoder(int level) {
    if (deflateInit(&zs_, level) != Z_OK) throw std::runtime_error("deflateInit failed");
}

ZrleEncoder::~ZrleEncoder() { deflateEnd(&zs_); }

void ZrleEncoder::encode_tile(const uint8_t* frame, size_t pitch, int x, int y, int w, int h, const int perm[3]) {
    const int n = w * h;
    px_.resize(n);
    for (int r = 0; r < h; ++r) {
        const uint8_t* row = frame + (size_t)(y + r) * pitch + (size_t)x * 4;
        for (int c = 0; c < w; ++c) {
            const uint8_t* p = row + 4 * c;
            px_[r * w + c] = (uint32_t)p[perm[0]] | ((uint32_t)p[perm[1]] << 8) | ((uint32_t)p[perm[2]] << 16);
        }
    }
    // palette (<= 16 colours, or give up) and run count
    uint32_t pal[16];
    int np = 0;
    bool pal_ok = true;
    int runs = 0, run_len_bytes = 0, pal_rle_bytes = 0;
    for (int i = 0; i < n;) {
        int j = i + 1;
        while (j < n && px_[j] == px_[i]) ++j;
        const int len = j - i;
        ++runs;
        run_len_bytes += run_bytes(len);
        pal_rle_bytes += (len == 1) ? 1 : 1 + run_bytes(len);
        if (pal_ok) {
            int k = 0;
            while (k < np && pal[k] != px_[i]) ++k;
            if (k == np) {
                if (np == 16) pal_ok = false;
                else pal[np++] = px_[i];
            }
        }
        i = j;
    }
    if (runs == 1) {  // solid
        raw_.push_back((char)1);
        put_cpixel(raw_, px_[0]);
        ++stats_[1];
        return;
    }
    const int raw_size = 3 * n;
    const int plain_rle = 3 * runs + run_len_bytes;
    int best = 0, best_size = raw_size;
    if (plain_rle < best_size) best = 128, best_size = plain_rle;
    int bits = 0;
    if (pal_ok) {
        bits = np <= 2 ? 1 : np <= 4 ? 2 : 4;
        const int packed = 3 * np + h * ((w * bits + 7) / 8);
        if (packed < best_size) best = np, best_size = packed;
        const int prle = 3 * np + pal_rle_bytes;
        if (prle < best_size) best = 128 + np, best_size = prle;
    }
    ++stats_[best];
    raw_.push_back((char)best);
    auto index_of = [&](uint32_t v) {
        int k = 0;
        while (pal[k] != v) ++k;
        return k;
    };
    if (best == 0) {
        for (int i = 0; i < n; ++i) put_cpixel(raw_, px_[i]);
    } else if (best == 128) {
        for (int i = 0; i < n;) {
            int j = i + 1;
            while (j < n && px_[j] == px_[i]) ++j;
            put_cpixel(raw_, px_[i]);
            put_run(raw_, j - i);
            i = j;
        }
    } else if (best > 128) {
        for (int k = 0; k < np; ++k) put_cpixel(raw_, pal[k]);
        for (int i = 0; i < n;) {
            int j = i + 1;
            while (j < n && px_[j] == px_[i]) ++j;
            const int idx = index_of(px_[i]);
            if (j - i == 1) {
                raw_.push_back((char)idx);
            } else {
                raw_.push_back((char)(idx | 128));
                put_run(raw_, j - i);
            }
            i = j;
        }
    } else {  // packed palette, rows padded to a byte, MSB first
        for (int k = 0; k < np; ++k) put_cpixel(raw_, pal[k]);
        for (int r = 0; r < h; ++r) {
            int acc = 0, nb = 0;
            for (int c = 0; c < w; ++c) {
                acc = (acc << bits) | index_of(px_[r * w + c]);
                nb += bits;
                if (nb == 8) {
                    raw_.push_back((char)acc);
                    acc = 0;
                    nb = 0;
                }
            }
            if (nb) raw_.push_back((char)(acc << (8 - nb)));
        }
    }
}

std::string ZrleEncoder::encode(const uint8_t* frame, size_t pitch, int x, int y, int w, int h, const int perm[3]) {
    for (int k = 0; k < 3; ++k)
        if (perm[k] < 0 || perm[k] > 3) throw std::invalid_argument("bad pixel permutation");
    raw_.clear();
    for (int ty = y; ty < y + h; ty += kTile)
        for (int tx = x; tx < x + w; tx += kTile)
            encode_tile(frame, pitch, tx, ty, std::min(kTile, x + w - tx), std::min(kTile, y + h - ty), perm);
    std::string out(4, '\0');
    std::vector<unsigned char> buf(deflateBound(&zs_, raw_.size()) + 64);
    zs_.next_in = (Bytef*)raw_.data();
    zs_.avail_in = (uInt)raw_.size();
    do {
        zs_.next_out = buf.data();
        zs_.avail_out = (uInt)buf.size();
        if (deflate(&zs_, Z_SYNC_FLUSH) == Z_STREAM_ERROR) throw std::runtime_error("deflate failed");
        out.append((const char*)buf.data(), buf.size() - zs_.avail_out);
    } while (zs_.avail_out == 0);
    const uint32_t len = (uint32_t)(out.size() - 4);
    out[0] = (char)(len >> 24);
    out[1] = (char)(len >> 16);
    out[2] = (char)(len >> 8);
    out[3] = (char)len;
    return out;
}

std::vector<uint8_t> tile_diff(const uint8_t* cur, const uint8_t* prev, size_t pitch, int w, int h, int tile) {
    const int tw = (w + tile - 1) / tile, th = (h + tile - 1) / tile;
    std::vector<uint8_t> flags((size_t)tw * th, 0);
    for (int ty = 0; ty < th; ++ty) {
        const int y0 = ty * tile, y1 = std::min(h, y0 + tile);
        for (int tx = 0; tx < tw; ++tx) {
            const int x0 = tx * tile, bytes = (std::min(w, x0 + tile) - x0) * 4;
            for (int y = y0; y < y1; ++y) {
                const size_t o = (size_t)y * pitch + (size_t)x0 * 4;
                if (std::memcmp(cur + o, prev + o, bytes) != 0) {
                    flags[(size_t)ty * tw + tx] = 1;
                    break;
                }
            }
        }
    }
    return flags;
}

}  // namespace rfb
}  // namespace mx
