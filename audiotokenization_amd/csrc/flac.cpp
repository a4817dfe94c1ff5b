// Host FLAC decoder (RFC 9639) for real-audio ingest: the reference reads LibriTTS / LibriSpeech .flac
// utterances through soundfile (extract_indices.py:98-106, `f.read(dtype='float32', always_2d=True)`), i.e.
// libsndfile over libFLAC, neither of which exists in this image.  This is a from-scratch decoder of the
// format, not a port of libFLAC: STREAMINFO, every subframe type (CONSTANT, VERBATIM, FIXED orders 0-4,
// LPC orders 1-32), Rice / escaped residual partitions (4- and 5-bit parameters), wasted bits, the
// left/side, side/right and mid/side decorrelations, fixed and variable block sizes, 4-32 bit samples,
// CRC-8 (frame header) and CRC-16 (frame) checks.  Output is planar [channel][sample], either the
// integers or float32 scaled by 2^-(bits-1) — libsndfile's normalised float read of integer FLAC.
// Host code only; the decoded clips go to the GPU resampler / encoder as float32 tensors.
#include <cstdint>
#include <cstring>
#include <vector>

namespace bc {
namespace {

enum FlacErr { FLAC_OK = 0, FLAC_EARG = 1, FLAC_ECORRUPT = 2, FLAC_EUNSUPPORTED = 3, FLAC_ECRC = 4, FLAC_ESPACE = 5 };

struct Bits {
  const uint8_t* p;
  uint64_t nbits;
  uint64_t pos = 0;
  bool bad = false;
  Bits(const uint8_t* d, uint64_t n) : p(d), nbits(n * 8) {}
  uint32_t u(int n) {  // n <= 32 bits, MSB first
    if (n == 0) return 0;
    if (pos + n > nbits) {
      bad = true;
      pos = nbits;
      return 0;
    }
    uint64_t v = 0;
    int got = 0;
    while (got < n) {
      const uint64_t byte = p[pos >> 3];
      const int off = pos & 7, avail = 8 - off, take = (n - got) < avail ? (n - got) : avail;
      v = (v << take) | ((byte >> (avail - take)) & ((1u << take) - 1));
      got += take;
      pos += take;
    }
    return (uint32_t)v;
  }
  int64_t s(int n) {  // two's complement, n <= 33
    if (n == 0) return 0;
    uint64_t v = n > 32 ? ((uint64_t)u(n - 32) << 32) | u(32) : u(n);
    if (v >> (n - 1)) v |= ~0ull << n;
    return (int64_t)v;
  }
  uint32_t unary() {  // zeros before the next one
    uint32_t z = 0;
    while (true) {
      if (pos >= nbits) {
        bad = true;
        return z;
      }
      const uint8_t byte = p[pos >> 3];
      const int off = pos & 7;
      const uint8_t rest = (uint8_t)(byte << off);
      if (rest) {
        const int lead = __builtin_clz((unsigned)rest) - 24;
        z += lead;
        pos += lead + 1;
        return z;
      }
      z += 8 - off;
      pos += 8 - off;
    }
  }
  void align() { pos = (pos + 7) & ~7ull; }
};

uint8_t crc8(const uint8_t* d, size_t n) {
  uint8_t c = 0;
  for (size_t i = 0; i < n; ++i) {
    c ^= d[i];
    for (int b = 0; b < 8; ++b) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : c << 1);
  }
  return c;
}

uint16_t crc16(const uint8_t* d, size_t n) {
  uint16_t c = 0;
  for (size_t i = 0; i < n; ++i) {
    c ^= (uint16_t)d[i] << 8;
    for (int b = 0; b < 8; ++b) c = (uint16_t)((c & 0x8000) ? (c << 1) ^ 0x8005 : c << 1);
  }
  return c;
}

struct StreamInfo {
  int min_block = 0, max_block = 0, rate = 0, channels = 0, bits = 0;
  uint64_t total = 0;
  uint64_t frames_pos = 0;  // byte offset of the first frame
};

int parse_header(const uint8_t* d, uint64_t n, StreamInfo& si) {
  if (n < 8 || memcmp(d, "fLaC", 4) != 0) return FLAC_ECORRUPT;
  uint64_t pos = 4;
  bool have = false;
  while (true) {
    if (pos + 4 > n) return FLAC_ECORRUPT;
    const bool last = d[pos] & 0x80;
    const int type = d[pos] & 0x7f;
    const uint32_t len = ((uint32_t)d[pos + 1] << 16) | ((uint32_t)d[pos + 2] << 8) | d[pos + 3];
    pos += 4;
    if (pos + len > n) return FLAC_ECORRUPT;
    if (type == 0) {
      if (len < 34) return FLAC_ECORRUPT;
      Bits b(d + pos, len);
      si.min_block = (int)b.u(16);
      si.max_block = (int)b.u(16);
      b.u(24);
      b.u(24);
      si.rate = (int)b.u(20);
      si.channels = (int)b.u(3) + 1;
      si.bits = (int)b.u(5) + 1;
      si.total = ((uint64_t)b.u(4) << 32) | b.u(32);
      have = true;
    } else if (type == 127) {
      return FLAC_ECORRUPT;
    }
    pos += len;
    if (last) break;
  }
  if (!have || si.bits < 4 || si.max_block < 16 || si.rate == 0) return FLAC_ECORRUPT;
  si.frames_pos = pos;
  return FLAC_OK;
}

// residual of one subframe into res[pred_order .. bs)
int read_residual(Bits& b, int bs, int order, int64_t* res) {
  const int method = (int)b.u(2);
  if (method > 1) return FLAC_ECORRUPT;
  const int pbits = method == 0 ? 4 : 5, esc = method == 0 ? 15 : 31;
  const int porder = (int)b.u(4);
  const int parts = 1 << porder;
  if ((bs >> porder) << porder != bs || (bs >> porder) < order) return FLAC_ECORRUPT;
  int i = order;
  for (int pt = 0; pt < parts; ++pt) {
    const int cnt = (bs >> porder) - (pt == 0 ? order : 0);
    const int k = (int)b.u(pbits);
    if (k == esc) {
      const int nb = (int)b.u(5);
      for (int j = 0; j < cnt; ++j) res[i++] = b.s(nb);
    } else {
      for (int j = 0; j < cnt; ++j) {
        const uint64_t q = b.unary();
        const uint64_t v = (q << k) | b.u(k);
        res[i++] = (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
      }
    }
    if (b.bad) return FLAC_ECORRUPT;
  }
  return FLAC_OK;
}

int read_subframe(Bits& b, int bs, int bps, int64_t* s) {
  if (b.u(1) != 0) return FLAC_ECORRUPT;
  const int type = (int)b.u(6);
  int wasted = 0;
  if (b.u(1)) wasted = (int)b.unary() + 1;
  if (wasted >= bps) return FLAC_ECORRUPT;
  bps -= wasted;
  if (type == 0) {  // CONSTANT
    const int64_t v = b.s(bps);
    for (int i = 0; i < bs; ++i) s[i] = v;
  } else if (type == 1) {  // VERBATIM
    for (int i = 0; i < bs; ++i) s[i] = b.s(bps);
  } else if (type >= 8 && type <= 12) {  // FIXED, order 0-4
    const int order = type - 8;
    if (order > bs) return FLAC_ECORRUPT;
    for (int i = 0; i < order; ++i) s[i] = b.s(bps);
    if (int rc = read_residual(b, bs, order, s)) return rc;
    for (int i = order; i < bs; ++i) {
      const int64_t r = s[i];
      switch (order) {
        case 0: break;
        case 1: s[i] = r + s[i - 1]; break;
        case 2: s[i] = r + 2 * s[i - 1] - s[i - 2]; break;
        case 3: s[i] = r + 3 * s[i - 1] - 3 * s[i - 2] + s[i - 3]; break;
        case 4: s[i] = r + 4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4]; break;
      }
    }
  } else if (type >= 32) {  // LPC, order 1-32
    const int order = type - 31;
    if (order > bs) return FLAC_ECORRUPT;
    for (int i = 0; i < order; ++i) s[i] = b.s(bps);
    const int prec = (int)b.u(4) + 1;
    if (prec == 16) return FLAC_ECORRUPT;
    const int shift = (int)b.s(5);
    if (shift < 0) return FLAC_EUNSUPPORTED;
    int64_t coef[32];
    for (int j = 0; j < order; ++j) coef[j] = b.s(prec);
    if (int rc = read_residual(b, bs, order, s)) return rc;
    for (int i = order; i < bs; ++i) {
      int64_t acc = 0;
      for (int j = 0; j < order; ++j) acc += coef[j] * s[i - 1 - j];
      s[i] += acc >> shift;
    }
  } else {
    return FLAC_ECORRUPT;  // reserved
  }
  if (b.bad) return FLAC_ECORRUPT;
  if (wasted)
    for (int i = 0; i < bs; ++i) s[i] = (int64_t)((uint64_t)s[i] << wasted);
  return FLAC_OK;
}

const int kRates[12] = {0, 88200, 176400, 192000, 8000, 16000, 22050, 24000, 32000, 44100, 48000, 96000};
const int kBits[8] = {0, 8, 12, -1, 16, 20, 24, 32};

// decode every frame; emit(channel, sample index, value) for each decoded sample (returns false = stop)
template <typename Emit>
long long decode_all(const uint8_t* d, uint64_t n, const StreamInfo& si, bool check_crc, Emit emit) {
  uint64_t pos = si.frames_pos;
  long long done = 0;
  std::vector<int64_t> ch[8];
  while (pos + 2 <= n) {
    if (d[pos] != 0xFF || (d[pos + 1] & 0xFC) != 0xF8) {  // not a frame start: trailing bytes (e.g. ID3) end the stream
      if (done == 0) return -FLAC_ECORRUPT;
      break;
    }
    Bits b(d + pos, n - pos);
    b.u(15);
    b.u(1);  // blocking strategy (the coded number's meaning only)
    const int bsc = (int)b.u(4), src = (int)b.u(4), chc = (int)b.u(4), ssc = (int)b.u(3);
    if (b.u(1) != 0) return -FLAC_ECORRUPT;
    // coded frame / sample number: UTF-8-like, 1-7 bytes
    const uint32_t first = b.u(8);
    int extra = 0;
    if (first & 0x80) {
      if ((first & 0xE0) == 0xC0) extra = 1;
      else if ((first & 0xF0) == 0xE0) extra = 2;
      else if ((first & 0xF8) == 0xF0) extra = 3;
      else if ((first & 0xFC) == 0xF8) extra = 4;
      else if ((first & 0xFE) == 0xFC) extra = 5;
      else if (first == 0xFE) extra = 6;
      else return -FLAC_ECORRUPT;
    }
    for (int i = 0; i < extra; ++i)
      if ((b.u(8) & 0xC0) != 0x80) return -FLAC_ECORRUPT;
    int bs;
    if (bsc == 0) return -FLAC_ECORRUPT;
    else if (bsc == 1) bs = 192;
    else if (bsc <= 5) bs = 576 << (bsc - 2);
    else if (bsc == 6) bs = (int)b.u(8) + 1;
    else if (bsc == 7) bs = (int)b.u(16) + 1;
    else bs = 256 << (bsc - 8);
    if (src == 12) b.u(8);
    else if (src == 13 || src == 14) b.u(16);
    else if (src == 15) return -FLAC_ECORRUPT;
    const int bps = ssc == 0 ? si.bits : kBits[ssc];
    if (bps <= 0) return -FLAC_ECORRUPT;
    if (b.bad) return -FLAC_ECORRUPT;
    const uint64_t hlen = b.pos >> 3;
    const uint8_t hcrc = (uint8_t)b.u(8);
    if (check_crc && crc8(d + pos, hlen) != hcrc) return -FLAC_ECRC;
    int nch;
    if (chc <= 7) nch = chc + 1;
    else if (chc <= 10) nch = 2;
    else return -FLAC_ECORRUPT;
    if (nch != si.channels) return -FLAC_ECORRUPT;
    for (int c = 0; c < nch; ++c) {
      ch[c].resize(bs);
      const bool side = (chc == 8 && c == 1) || (chc == 9 && c == 0) || (chc == 10 && c == 1);
      if (int rc = read_subframe(b, bs, bps + (side ? 1 : 0), ch[c].data())) return -rc;
    }
    b.align();
    const uint64_t flen = b.pos >> 3;
    const uint16_t fcrc = (uint16_t)b.u(16);
    if (b.bad) return -FLAC_ECORRUPT;
    if (check_crc && crc16(d + pos, flen) != fcrc) return -FLAC_ECRC;
    if (chc == 8) {  // left / side
      for (int i = 0; i < bs; ++i) ch[1][i] = ch[0][i] - ch[1][i];
    } else if (chc == 9) {  // side / right
      for (int i = 0; i < bs; ++i) ch[0][i] += ch[1][i];
    } else if (chc == 10) {  // mid / side
      for (int i = 0; i < bs; ++i) {
        const int64_t side = ch[1][i];
        const int64_t mid = ((uint64_t)ch[0][i] << 1) | (side & 1);
        ch[0][i] = (mid + side) >> 1;
        ch[1][i] = (mid - side) >> 1;
      }
    }
    for (int c = 0; c < nch; ++c)
      for (int i = 0; i < bs; ++i)
        if (!emit(c, done + i, ch[c][i])) return -FLAC_ESPACE;
    done += bs;
    pos += flen + 2;
  }
  if (si.total && (uint64_t)done != si.total) return -FLAC_ECORRUPT;
  return done;
}

}  // namespace
}  // namespace bc

extern "C" {

int bc_flac_info(const unsigned char* data, long long n, int* sample_rate, int* channels, int* bits,
                 long long* total_samples) {
  if (!data || n <= 0) return bc::FLAC_EARG;
  bc::StreamInfo si;
  if (int rc = bc::parse_header(data, (uint64_t)n, si)) return rc;
  if (sample_rate) *sample_rate = si.rate;
  if (channels) *channels = si.channels;
  if (bits) *bits = si.bits;
  if (total_samples) *total_samples = (long long)si.total;
  return 0;
}

long long bc_flac_decode(const unsigned char* data, long long n, void* out, int out_int32, long long max_samples,
                         int check_crc) {
  if (!data || n <= 0 || !out || max_samples < 0) return -bc::FLAC_EARG;
  bc::StreamInfo si;
  if (int rc = bc::parse_header(data, (uint64_t)n, si)) return -rc;
  const int C = si.channels;
  if (out_int32) {
    int32_t* o = static_cast<int32_t*>(out);
    return bc::decode_all(data, (uint64_t)n, si, check_crc != 0, [&](int c, long long i, int64_t v) {
      if (i >= max_samples) return false;
      o[(long long)c * max_samples + i] = (int32_t)v;
      return true;
    });
  }
  float* o = static_cast<float*>(out);
  const double scale = 1.0 / (double)(1ull << (si.bits - 1));
  (void)C;
  return bc::decode_all(data, (uint64_t)n, si, check_crc != 0, [&](int c, long long i, int64_t v) {
    if (i >= max_samples) return false;
    o[(long long)c * max_samples + i] = (float)((double)v * scale);
    return true;
  });
}

}  // extern "C"
