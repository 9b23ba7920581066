// Host reads of the drop-in integrate: per frame, the raw NDC depth file
// (H*W little-endian float32; reference dataio/depth_data_io.py:33-53 via np.fromfile) and the confidence
// npz written by np.savez (members confidence_map <f8 HxW and valid_count <i4 HxW;
// depth_data_io.py:91-115), read by native threads with pread straight into the caller's arrays.
//
// np.savez stores members uncompressed, so each member's array bytes are one contiguous file range:
// the zip central directory gives the member's local header, the local header its data start, the .npy
// header the dtype / order / shape and the data offset.  Anything else -- a compressed or otherwise
// unexpected archive, another dtype or shape, a raw file of the wrong size, a read error -- is reported
// per frame and left to the caller's own loader, so error behaviour stays the reference's.
// Round 5: the Python loader (np.load per npz on 8 I/O threads) bounded the drop-in integrate at
// 0.28-0.53 s of waiting per 500-frame call against 0.05-0.08 s of device hand-off (bench
// dropin_e2e.integrate_splits_s).
#include <fcntl.h>
#include <immintrin.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <string>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "mqr_common.hpp"

namespace {

struct Fd {
    int fd = -1;
    explicit Fd(const char* p) : fd(::open(p, O_RDONLY | O_CLOEXEC)) {}
    ~Fd() {
        if (fd >= 0) ::close(fd);
    }
};

bool pread_all(int fd, void* dst, size_t n, int64_t off) {
    char* p = static_cast<char*>(dst);
    while (n) {
        const ssize_t r = ::pread(fd, p, n, (off_t)off);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        p += r;
        n -= (size_t)r;
        off += r;
    }
    return true;
}

uint16_t u16(const unsigned char* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
uint32_t u32(const unsigned char* p) { return (uint32_t)u16(p) | ((uint32_t)u16(p + 2) << 16); }
uint64_t u64(const unsigned char* p) { return (uint64_t)u32(p) | ((uint64_t)u32(p + 4) << 32); }

// The .npy header dict: {'descr': '<f8', 'fortran_order': False, 'shape': (H, W), }
bool npy_header_ok(const std::string& h, const char* descr, int H, int W) {
    auto value_after = [&](const char* key) -> std::string {
        const size_t k = h.find(key);
        if (k == std::string::npos) return "";
        size_t c = h.find(':', k);
        if (c == std::string::npos) return "";
        ++c;
        while (c < h.size() && h[c] == ' ') ++c;
        return h.substr(c);
    };
    const std::string d = value_after("'descr'");
    if (d.compare(0, strlen(descr) + 2, std::string("'") + descr + "'") != 0) return false;
    if (value_after("'fortran_order'").compare(0, 5, "False") != 0) return false;
    const std::string s = value_after("'shape'");
    long a = -1, b = -1;
    if (s.empty() || s[0] != '(' || sscanf(s.c_str(), "(%ld, %ld)", &a, &b) != 2) return false;
    const size_t close = s.find(')');
    return close != std::string::npos && a == H && b == W &&
           std::count(s.begin(), s.begin() + (std::ptrdiff_t)close, ',') == 1;
}

// Locate the array bytes of member `name` (stored) in the zip at fd: file offset of the data, or -1.
struct Member {
    std::string name;
    int64_t data_off = -1;
    int64_t size = -1;
};

bool zip_members(int fd, int64_t fsize, std::vector<Member>& want) {
    // end of central directory: the last 22..(22 + 65535) bytes
    const int64_t tail = std::min<int64_t>(fsize, 22 + 65535);
    std::vector<unsigned char> t((size_t)tail);
    if (!pread_all(fd, t.data(), t.size(), fsize - tail)) return false;
    int64_t e = -1;
    for (int64_t i = tail - 22; i >= 0; --i)
        if (u32(&t[(size_t)i]) == 0x06054b50u) {
            e = i;
            break;
        }
    if (e < 0) return false;
    uint64_t entries = u16(&t[(size_t)e + 10]), cd_size = u32(&t[(size_t)e + 12]), cd_off = u32(&t[(size_t)e + 16]);
    if (entries == 0xFFFF || cd_size == 0xFFFFFFFFu || cd_off == 0xFFFFFFFFu) {  // zip64 end record
        if (e < 20 || u32(&t[(size_t)e - 20]) != 0x07064b50u) return false;
        const uint64_t z64 = u64(&t[(size_t)e - 20 + 8]);
        unsigned char r[56];
        if (!pread_all(fd, r, sizeof r, (int64_t)z64) || u32(r) != 0x06064b50u) return false;
        entries = u64(r + 32);
        cd_size = u64(r + 40);
        cd_off = u64(r + 48);
    }
    if (cd_off + cd_size > (uint64_t)fsize || cd_size > (uint64_t(1) << 24)) return false;
    std::vector<unsigned char> cd((size_t)cd_size);
    if (!pread_all(fd, cd.data(), cd.size(), (int64_t)cd_off)) return false;
    size_t p = 0;
    for (uint64_t k = 0; k < entries; ++k) {
        if (p + 46 > cd.size() || u32(&cd[p]) != 0x02014b50u) return false;
        const uint16_t method = u16(&cd[p + 10]), nlen = u16(&cd[p + 28]), xlen = u16(&cd[p + 30]),
                       clen = u16(&cd[p + 32]);
        uint64_t csize = u32(&cd[p + 20]), usize = u32(&cd[p + 24]), loff = u32(&cd[p + 42]);
        if (p + 46 + nlen + xlen + clen > cd.size()) return false;
        const std::string name(reinterpret_cast<const char*>(&cd[p + 46]), nlen);
        // zip64 extra field: the 0xFFFFFFFF fields, in order usize, csize, offset
        for (size_t x = p + 46 + nlen; x + 4 <= p + 46 + nlen + xlen;) {
            const uint16_t id = u16(&cd[x]), len = u16(&cd[x + 2]);
            if (id == 0x0001) {
                size_t q = x + 4;
                if (usize == 0xFFFFFFFFu && q + 8 <= x + 4 + len) usize = u64(&cd[q]), q += 8;
                if (csize == 0xFFFFFFFFu && q + 8 <= x + 4 + len) csize = u64(&cd[q]), q += 8;
                if (loff == 0xFFFFFFFFu && q + 8 <= x + 4 + len) loff = u64(&cd[q]), q += 8;
            }
            x += 4 + len;
        }
        for (Member& m : want)
            if (m.name == name) {
                if (method != 0 || csize != usize) return false;  // compressed (np.savez_compressed)
                unsigned char lh[30];
                if (!pread_all(fd, lh, sizeof lh, (int64_t)loff) || u32(lh) != 0x04034b50u) return false;
                m.data_off = (int64_t)loff + 30 + u16(lh + 26) + u16(lh + 28);
                m.size = (int64_t)usize;
            }
        p += 46 + nlen + xlen + clen;
    }
    for (const Member& m : want)
        if (m.data_off < 0 || m.data_off + m.size > fsize) return false;
    return true;
}

// The file offset of the array bytes of one .npy member at [off, off + size) after checking its header
// (dtype, C order, shape H x W, size), or -1.
int64_t npy_data_off(int fd, const Member& m, const char* descr, size_t item, int H, int W) {
    unsigned char pre[12];
    if (m.size < 10 || !pread_all(fd, pre, 10, m.data_off)) return -1;
    if (memcmp(pre, "\x93NUMPY", 6) != 0) return -1;
    int64_t hl, hoff;
    if (pre[6] == 1) {
        hl = u16(pre + 8);
        hoff = 10;
    } else if (pre[6] == 2 || pre[6] == 3) {
        if (m.size < 12 || !pread_all(fd, pre, 12, m.data_off)) return -1;
        hl = u32(pre + 8);
        hoff = 12;
    } else {
        return -1;
    }
    const size_t bytes = item * (size_t)H * (size_t)W;
    if (hl > 65536 || hoff + hl + (int64_t)bytes != m.size) return -1;
    std::string h((size_t)hl, '\0');
    if (!pread_all(fd, &h[0], (size_t)hl, m.data_off + hoff)) return -1;
    if (!npy_header_ok(h, descr, H, W)) return -1;
    return m.data_off + hoff + hl;
}

// Reads the H*W*item array bytes of one .npy member into dst.
bool read_npy(int fd, const Member& m, const char* descr, size_t item, int H, int W, void* dst) {
    const int64_t off = npy_data_off(fd, m, descr, item, H, W);
    return off >= 0 && pread_all(fd, dst, item * (size_t)H * (size_t)W, off);
}

// The confidence mask of one frame, one byte per pixel: (confidence_map < conf_thr) | (valid_count <
// count_thr), the comparison the decode applies (ingest.hip decode_px; reference o3d_utils.py:47-50 via
// dataio/depth_data_io.py:125-131).  Both members are read in blocks through a thread-local buffer.
bool read_mask(int fd, const Member* m, int H, int W, double conf_thr, int count_thr, uint8_t* mask) {
    const size_t HW = (size_t)H * (size_t)W;
    const int64_t oc = npy_data_off(fd, m[0], "<f8", 8, H, W), ov = npy_data_off(fd, m[1], "<i4", 4, H, W);
    if (oc < 0 || ov < 0) return false;
    constexpr size_t kBlock = 32768;  // pixels per read: 256 KiB of confidence
    thread_local std::vector<double> cb(kBlock);
    thread_local std::vector<int32_t> vb(kBlock);
    for (size_t p = 0; p < HW; p += kBlock) {
        const size_t k = std::min(kBlock, HW - p);
        if (!pread_all(fd, cb.data(), 8 * k, oc + 8 * (int64_t)p) ||
            !pread_all(fd, vb.data(), 4 * k, ov + 4 * (int64_t)p))
            return false;
        for (size_t i = 0; i < k; ++i) mask[p + i] = (uint8_t)((int)(cb[i] < conf_thr) | (int)(vb[i] < count_thr));
    }
    return true;
}

// CRC-32 (zip / gzip polynomial, reflected) by carry-less multiplication: four 128-bit lanes folded
// 64 bytes at a time, folded to 128 bits, then 64, then Barrett-reduced (Gopal et al., "Fast CRC
// Computation for Generic Polynomials Using PCLMULQDQ Instruction", Intel 2009; constants x^k mod P for
// the bit-reflected P = 0x104C11DB7).  len >= 64 and a multiple of 16; crc in and out pre-inverted.
#define MQR_CLMUL __attribute__((target("pclmul,sse4.1"), always_inline)) inline
MQR_CLMUL __m128i ld(const unsigned char* q) { return _mm_loadu_si128(reinterpret_cast<const __m128i*>(q)); }
MQR_CLMUL __m128i fold(__m128i a, __m128i k, __m128i next) {
    return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(a, k, 0x11), _mm_clmulepi64_si128(a, k, 0x00)), next);
}

__attribute__((target("pclmul,sse4.1"))) uint32_t crc32_fold(const unsigned char* p, size_t len, uint32_t crc) {
    alignas(16) static const uint64_t k12[2] = {0x0154442bd4ull, 0x01c6e41596ull};
    alignas(16) static const uint64_t k34[2] = {0x01751997d0ull, 0x00ccaa009eull};
    alignas(16) static const uint64_t k50[2] = {0x0163cd6124ull, 0ull};
    alignas(16) static const uint64_t pmu[2] = {0x01db710641ull, 0x01f7011641ull};
    __m128i a0 = _mm_xor_si128(ld(p), _mm_cvtsi32_si128((int)crc)), a1 = ld(p + 16), a2 = ld(p + 32), a3 = ld(p + 48);
    __m128i k = _mm_load_si128(reinterpret_cast<const __m128i*>(k12));
    p += 64;
    len -= 64;
    for (; len >= 64; p += 64, len -= 64) {
        a0 = fold(a0, k, ld(p));
        a1 = fold(a1, k, ld(p + 16));
        a2 = fold(a2, k, ld(p + 32));
        a3 = fold(a3, k, ld(p + 48));
    }
    k = _mm_load_si128(reinterpret_cast<const __m128i*>(k34));
    a0 = fold(a0, k, a1);
    a0 = fold(a0, k, a2);
    a0 = fold(a0, k, a3);
    for (; len >= 16; p += 16, len -= 16) a0 = fold(a0, k, ld(p));
    const __m128i lo32 = _mm_setr_epi32(-1, 0, -1, 0);
    __m128i t = _mm_clmulepi64_si128(a0, k, 0x10);  // 128 -> 64 bits
    a0 = _mm_xor_si128(_mm_srli_si128(a0, 8), t);
    k = _mm_loadl_epi64(reinterpret_cast<const __m128i*>(k50));
    t = _mm_srli_si128(a0, 4);
    a0 = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(a0, lo32), k, 0x00), t);
    k = _mm_load_si128(reinterpret_cast<const __m128i*>(pmu));  // Barrett reduction to 32 bits
    t = _mm_clmulepi64_si128(_mm_and_si128(a0, lo32), k, 0x10);
    t = _mm_clmulepi64_si128(_mm_and_si128(t, lo32), k, 0x00);
    return (uint32_t)_mm_extract_epi32(_mm_xor_si128(a0, t), 1);
}

uint32_t crc32_of(uint32_t crc, const void* data, size_t len) {
    const unsigned char* p = static_cast<const unsigned char*>(data);
    if (len >= 64 && __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1")) {
        const size_t body = len & ~(size_t)15;
        crc = ~crc32_fold(p, body, ~crc);
        p += body;
        len -= body;
    }
    while (len) {  // zlib for the tail (and without PCLMULQDQ)
        const uInt n = (uInt)std::min<size_t>(len, 1u << 30);
        crc = (uint32_t)crc32(crc, p, n);
        p += n;
        len -= n;
    }
    return crc;
}

bool pwrite_all(int fd, const void* src, size_t n, int64_t off) {
    const char* p = static_cast<const char*>(src);
    while (n) {
        const ssize_t r = ::pwrite(fd, p, n, (off_t)off);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        p += r;
        n -= (size_t)r;
        off += r;
    }
    return true;
}

void put16(std::string& s, uint16_t v) { s.push_back((char)(v & 0xFF)), s.push_back((char)(v >> 8)); }
void put32(std::string& s, uint32_t v) { put16(s, (uint16_t)(v & 0xFFFF)), put16(s, (uint16_t)(v >> 16)); }
void put64(std::string& s, uint64_t v) { put32(s, (uint32_t)(v & 0xFFFFFFFFu)), put32(s, (uint32_t)(v >> 32)); }

// .npy format 1.0 header of a C-order H x W array, padded with spaces to a 64-byte multiple (numpy's
// ARRAY_ALIGN) and ended by a newline
std::string npy_header(const char* descr, int H, int W) {
    std::string d = std::string("{'descr': '") + descr + "', 'fortran_order': False, 'shape': (" + std::to_string(H) +
                    ", " + std::to_string(W) + "), }";
    const size_t total = (10 + d.size() + 1 + 63) / 64 * 64;
    d.append(total - 10 - d.size() - 1, ' ');
    d.push_back('\n');
    std::string h("\x93NUMPY\x01\x00", 8);
    put16(h, (uint16_t)d.size());
    return h + d;
}

// One np.savez-layout npz: stored members in the given order, each a local header with a zip64 extra
// field (np.savez opens its members with force_zip64), then the central directory and end record.
// A member's array bytes come from `data`, or, when `fill` is set, are produced block by block: fill(off, n,
// dst) writes bytes [off, off + n) of the array to dst (whole items), each block checksummed and written
// while it is in cache.
struct NpzMember {
    const char* name;
    std::string npy;  // .npy header
    const void* data;
    size_t bytes;
    std::function<void(size_t, size_t, void*)> fill = nullptr;
};

// The CRC of the header + array of member m, written at data_off (the array) -- from the caller's bytes or
// through fill's blocks.
bool put_member_data(int fd, const NpzMember& m, int64_t data_off, uint32_t& crc) {
    crc = crc32_of(0, m.npy.data(), m.npy.size());
    if (!m.fill) {
        crc = crc32_of(crc, m.data, m.bytes);
        return pwrite_all(fd, m.data, m.bytes, data_off);
    }
    constexpr size_t kBlock = size_t(1) << 17;
    thread_local std::vector<uint64_t> blk(kBlock / 8);
    for (size_t o = 0; o < m.bytes; o += kBlock) {
        const size_t k = std::min(kBlock, m.bytes - o);
        m.fill(o, k, blk.data());
        crc = crc32_of(crc, blk.data(), k);
        if (!pwrite_all(fd, blk.data(), k, data_off + (int64_t)o)) return false;
    }
    return true;
}

int write_npz(const char* path, NpzMember* m, int nm) {
    const int fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) return errno ? errno : EIO;
    // the array bytes first (their CRCs go into the headers), then the headers, directory and end record
    int64_t off = 0;
    std::vector<int64_t> lh_off(nm);
    std::vector<uint32_t> crc(nm);
    std::vector<std::string> lh(nm);
    bool ok = true;
    for (int i = 0; i < nm; ++i) {
        lh_off[i] = off;
        const size_t lh_size = 30 + strlen(m[i].name) + 20;
        ok = ok && put_member_data(fd, m[i], off + (int64_t)(lh_size + m[i].npy.size()), crc[i]);
        off += (int64_t)(lh_size + m[i].npy.size() + m[i].bytes);
    }
    for (int i = 0; i < nm; ++i) {
        const uint64_t size = m[i].npy.size() + m[i].bytes;
        std::string& h = lh[i];
        put32(h, 0x04034b50u);
        put16(h, 45);  // version needed: zip64
        put16(h, 0);   // flags
        put16(h, 0);   // stored
        put16(h, 0);   // time
        put16(h, (1 << 5) | 1);  // date 1980-01-01
        put32(h, crc[i]);
        put32(h, 0xFFFFFFFFu);
        put32(h, 0xFFFFFFFFu);
        put16(h, (uint16_t)strlen(m[i].name));
        put16(h, 20);
        h += m[i].name;
        put16(h, 0x0001);
        put16(h, 16);
        put64(h, size);
        put64(h, size);
    }
    std::string cd;
    for (int i = 0; i < nm; ++i) {
        const uint64_t size = m[i].npy.size() + m[i].bytes;
        const bool big = size >= 0xFFFFFFFFull || (uint64_t)lh_off[i] >= 0xFFFFFFFFull;
        put32(cd, 0x02014b50u);
        put16(cd, 45);
        put16(cd, 45);
        put16(cd, 0);
        put16(cd, 0);
        put16(cd, 0);
        put16(cd, (1 << 5) | 1);
        put32(cd, crc[i]);
        put32(cd, big ? 0xFFFFFFFFu : (uint32_t)size);
        put32(cd, big ? 0xFFFFFFFFu : (uint32_t)size);
        put16(cd, (uint16_t)strlen(m[i].name));
        put16(cd, big ? 28 : 0);
        put16(cd, 0);  // comment
        put16(cd, 0);  // disk
        put16(cd, 0);  // internal attributes
        put32(cd, 0600u << 16);  // external attributes (unix mode, as zipfile writes them)
        put32(cd, big ? 0xFFFFFFFFu : (uint32_t)lh_off[i]);
        cd += m[i].name;
        if (big) {
            put16(cd, 0x0001);
            put16(cd, 24);
            put64(cd, size);
            put64(cd, size);
            put64(cd, (uint64_t)lh_off[i]);
        }
    }
    const int64_t cd_off = off;
    std::string end;
    if (cd_off >= 0xFFFFFFFFll) {  // zip64 end record + locator
        put32(end, 0x06064b50u);
        put64(end, 44);
        put16(end, 45);
        put16(end, 45);
        put32(end, 0);
        put32(end, 0);
        put64(end, (uint64_t)nm);
        put64(end, (uint64_t)nm);
        put64(end, cd.size());
        put64(end, (uint64_t)cd_off);
        put32(end, 0x07064b50u);
        put32(end, 0);
        put64(end, (uint64_t)(cd_off + (int64_t)cd.size()));
        put32(end, 1);
    }
    put32(end, 0x06054b50u);
    put16(end, 0);
    put16(end, 0);
    put16(end, (uint16_t)nm);
    put16(end, (uint16_t)nm);
    put32(end, (uint32_t)cd.size());
    put32(end, cd_off >= 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)cd_off);
    put16(end, 0);
    for (int i = 0; i < nm && ok; ++i) {
        ok = pwrite_all(fd, lh[i].data(), lh[i].size(), lh_off[i]) &&
             pwrite_all(fd, m[i].npy.data(), m[i].npy.size(), lh_off[i] + (int64_t)lh[i].size());
    }
    ok = ok && pwrite_all(fd, cd.data(), cd.size(), cd_off) &&
         pwrite_all(fd, end.data(), end.size(), cd_off + (int64_t)cd.size());
    const int err = ok ? 0 : (errno ? errno : EIO);
    if (::close(fd) != 0 && ok) return errno ? errno : EIO;
    return err;
}

}  // namespace

extern "C" {

uint32_t mqr_crc32(uint32_t crc, const void* data, int64_t len) { return len > 0 ? crc32_of(crc, data, (size_t)len) : crc; }

int mqr_write_confidence_npz(int n, const char* const* paths, const double* conf, const int32_t* valid, int H, int W,
                             int32_t* status, int threads) {
    MQR_REQUIRE(n >= 0 && H > 0 && W > 0, "bad sizes");
    MQR_REQUIRE(n == 0 || (paths && conf && valid && status), "null argument");
    const size_t HW = (size_t)H * (size_t)W;
    const std::string h_conf = npy_header("<f8", H, W), h_valid = npy_header("<i4", H, W);
    std::atomic<int> next{0};
    auto work = [&] {
        for (int f; (f = next.fetch_add(1)) < n;) {
            NpzMember m[2] = {{"confidence_map.npy", h_conf, conf + (size_t)f * HW, 8 * HW},
                              {"valid_count.npy", h_valid, valid + (size_t)f * HW, 4 * HW}};
            status[f] = paths[f] ? write_npz(paths[f], m, 2) : 0;  // null path: no file for this frame
        }
    };
    const int T = std::max(1, std::min({threads > 0 ? threads : 8, 64, std::max(n, 1)}));
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
    return 0;
}


// Both readers: the maps themselves (conf_out / vc_out) or the mask byte per pixel (mask_out).
static int read_frames(int n, const char* const* raw_paths, const char* const* conf_paths, int H, int W,
                       float* raw_out, double* conf_out, int32_t* vc_out, uint8_t* mask_out, double conf_thr,
                       int count_thr, uint8_t* status, int threads) {
    MQR_REQUIRE(n >= 0 && H > 0 && W > 0, "bad sizes");
    MQR_REQUIRE(n == 0 || (raw_paths && raw_out && status), "null argument");
    const size_t HW = (size_t)H * (size_t)W;
    std::atomic<int> next{0};
    auto work = [&] {
        for (int f; (f = next.fetch_add(1)) < n;) {
            uint8_t st = 0;
            float* raw = raw_out + (size_t)f * HW;
            {
                Fd fd(raw_paths[f]);
                struct stat sb {};
                if (fd.fd < 0) {
                    st |= errno == ENOENT ? MQR_FRAME_RAW_MISSING : MQR_FRAME_RAW_OTHER;
                } else if (fstat(fd.fd, &sb) != 0 || (size_t)sb.st_size != 4 * HW || !pread_all(fd.fd, raw, 4 * HW, 0)) {
                    st |= MQR_FRAME_RAW_OTHER;
                } else {
                    st |= MQR_FRAME_RAW_OK;
                }
                if (!(st & MQR_FRAME_RAW_OK)) memset(raw, 0, 4 * HW);  // no frame: zeros, decoded invalid
            }
            if (conf_paths && conf_paths[f]) {
                Fd fd(conf_paths[f]);
                struct stat sb {};
                if (fd.fd < 0) {
                    st |= errno == ENOENT ? MQR_FRAME_CONF_MISSING : MQR_FRAME_CONF_OTHER;
                } else {
                    std::vector<Member> m(2);
                    m[0].name = "confidence_map.npy";
                    m[1].name = "valid_count.npy";
                    const bool ok = fstat(fd.fd, &sb) == 0 && zip_members(fd.fd, sb.st_size, m) &&
                                    (mask_out ? read_mask(fd.fd, m.data(), H, W, conf_thr, count_thr,
                                                          mask_out + (size_t)f * HW)
                                              : read_npy(fd.fd, m[0], "<f8", 8, H, W, conf_out + (size_t)f * HW) &&
                                                    read_npy(fd.fd, m[1], "<i4", 4, H, W, vc_out + (size_t)f * HW));
                    st |= ok ? MQR_FRAME_CONF_OK : MQR_FRAME_CONF_OTHER;
                }
            }
            status[f] = st;
        }
    };
    const int T = std::max(1, std::min({threads > 0 ? threads : 8, 64, std::max(n, 1)}));
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
    return 0;
}

int mqr_write_confidence_npz_counts(int n, const char* const* paths, const uint16_t* counts, int H, int W,
                                    int32_t* status, int threads) {
    MQR_REQUIRE(n >= 0 && H > 0 && W > 0, "bad sizes");
    MQR_REQUIRE(n == 0 || (paths && counts && status), "null argument");
    // confidence_map of a (valid, consistent) pair: np.true_divide(consistent, valid) -- the correctly
    // rounded float64 quotient -- and 0 where valid is 0 (estimate_depth_confidences.py:72-74)
    static double table[1 << 16];
    static std::once_flag once;
    std::call_once(once, [] {
        for (int c = 0; c < (1 << 16); ++c) {
            const int v = c & 0xFF, k = c >> 8;
            table[c] = v ? (double)k / (double)v : 0.0;
        }
    });
    const size_t HW = (size_t)H * (size_t)W;
    const std::string h_conf = npy_header("<f8", H, W), h_valid = npy_header("<i4", H, W);
    std::atomic<int> next{0};
    auto work = [&] {
        for (int f; (f = next.fetch_add(1)) < n;) {
            if (!paths[f]) {
                status[f] = 0;
                continue;
            }
            const uint16_t* c = counts + (size_t)f * HW;
            // the maps expanded block by block into the writer's cache-resident buffer
            NpzMember m[2] = {{"confidence_map.npy", h_conf, nullptr, 8 * HW,
                               [c](size_t off, size_t nb, void* dst) {
                                   double* d = static_cast<double*>(dst);
                                   const uint16_t* s = c + off / 8;
                                   for (size_t i = 0; i < nb / 8; ++i) d[i] = table[s[i]];
                               }},
                              {"valid_count.npy", h_valid, nullptr, 4 * HW, [c](size_t off, size_t nb, void* dst) {
                                   int32_t* d = static_cast<int32_t*>(dst);
                                   const uint16_t* s = c + off / 4;
                                   for (size_t i = 0; i < nb / 4; ++i) d[i] = s[i] & 0xFF;
                               }}};
            status[f] = write_npz(paths[f], m, 2);
        }
    };
    const int T = std::max(1, std::min({threads > 0 ? threads : 8, 64, std::max(n, 1)}));
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
    return 0;
}

int mqr_read_frames(int n, const char* const* raw_paths, const char* const* conf_paths, int H, int W, float* raw_out,
                    double* conf_out, int32_t* vc_out, uint8_t* status, int threads) {
    MQR_REQUIRE(!conf_paths || (conf_out && vc_out), "confidence paths without output arrays");
    return read_frames(n, raw_paths, conf_paths, H, W, raw_out, conf_out, vc_out, nullptr, 0.0, 0, status, threads);
}

int mqr_read_frames_masked(int n, const char* const* raw_paths, const char* const* conf_paths, int H, int W,
                           double conf_thr, int count_thr, float* raw_out, uint8_t* mask_out, uint8_t* status,
                           int threads) {
    MQR_REQUIRE(!conf_paths || mask_out, "confidence paths without a mask array");
    return read_frames(n, raw_paths, conf_paths, H, W, raw_out, nullptr, nullptr, mask_out, conf_thr, count_thr,
                       status, threads);
}

}  // extern "C"
