// pt_jpeg.cpp — JPEG decode for the hosts' texture loading: the glTF models' PBR maps arrive as
// JPEG bytes (the glTF loader's textures, js/GLTF_Model_Path_Tracing.js:252-274; `new
// BABYLON.Texture(url)` decodes them in the browser). Both hosts decode here, so the Node host
// needs no Python and the two hosts upload the same texels.
//
// The decoder a browser uses is not pinned; this one reproduces libjpeg-turbo's default
// decompression exactly (what Pillow and Chromium use): baseline and progressive Huffman scans,
// the accurate integer IDCT (jidctint.c jpeg_idct_islow, with its post-IDCT range-limit table),
// "fancy" triangle-filter chroma upsampling (jdsample.c h2v1 / h1v2 / h2v2, edge rows and columns
// replicated) and the fixed-point YCbCr -> RGB tables (jdcolor.c). Arithmetic coding, 12-bit
// samples, CMYK / Adobe-transform files are refused (PT_ERR_UNSUPPORTED). Host code only.
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/pt.h"

namespace {

const int kZigzag[64 + 16] = {   // jpeg_natural_order (+ 16 entries of 63 for corrupt runs)
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63 };

struct Huff {
    bool present = false;
    int maxcode[18];       // largest code of length l (-1: none); maxcode[17] sentinel
    int valoff[17];        // symbol index offset for length l
    uint8_t vals[256];
    uint16_t look[256];    // 8-bit lookahead: (length << 8) | symbol, 0 = longer code
};

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0;
    int bw = 0, bh = 0;      // blocks of the component proper (ceil(dw / 8) x ceil(dh / 8))
    int bwm = 0, bhm = 0;    // blocks of the MCU-padded grid
    int dw = 0, dh = 0;      // downsampled size: ceil(W * h / hmax) x ceil(H * v / vmax)
    int td = 0, ta = 0, dcpred = 0;
    std::vector<int16_t> coef;   // bwm * bhm blocks x 64, natural order
};

struct Decoder {
    const uint8_t* p;
    const uint8_t* end;
    int W = 0, H = 0, ncomp = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    bool progressive = false, seenSof = false, adobe = false;
    int adobeTransform = -1;
    int restart = 0;
    uint16_t q[4][64] = {};   // natural order
    bool qset[4] = {};        // tables a DQT segment defined
    Huff dc[4], ac[4];
    Comp c[4];
    // bit reader (F.2.2.5): 0xFF00 -> 0xFF; a marker ends the entropy data (zeros are fed after it)
    uint32_t acc = 0;
    int nbits = 0;
    bool hitMarker = false;
    int eobrun = 0;

    int u8() { return p < end ? *p++ : -1; }
    int u16() { const int a = u8(), b = u8(); return (a < 0 || b < 0) ? -1 : (a << 8) | b; }

    void fill()
    {
        while (nbits <= 24) {
            int b = 0;
            if (!hitMarker && p < end) {
                b = *p;
                if (b == 0xFF) {
                    const int n = p + 1 < end ? p[1] : 0xD9;
                    if (n == 0x00) p += 2;
                    else { hitMarker = true; b = 0; }   // leave the marker for the parser
                } else p++;
            }
            acc |= (uint32_t)b << (24 - nbits);
            nbits += 8;
        }
    }
    int bits(int n)
    {
        if (n == 0) return 0;
        fill();
        const int v = (int)(acc >> (32 - n));
        acc <<= n; nbits -= n;
        return v;
    }
    int bit() { return bits(1); }
    int decode(const Huff& t)
    {
        fill();
        const uint16_t e = t.look[acc >> 24];
        if (e) { const int l = e >> 8; acc <<= l; nbits -= l; return e & 255; }
        int code = (int)(acc >> 24), l = 8;
        acc <<= 8; nbits -= 8;
        while (l < 16 && code > t.maxcode[l]) { code = (code << 1) | bits(1); l++; }
        if (code > t.maxcode[l]) return 0;   // corrupt: libjpeg substitutes a zero symbol
        return t.vals[(t.valoff[l] + code) & 255];
    }
    static int extend(int v, int s) { return v < (1 << (s - 1)) ? v + (int)((-1u) << s) + 1 : v; }
    void resetBits() { acc = 0; nbits = 0; hitMarker = false; }

    int readHuff(int len)
    {
        while (len > 0) {
            const int tc = u8();
            if (tc < 0) return PT_ERR_DATA;
            const int cls = tc >> 4, id = tc & 15;
            if (cls > 1 || id > 3) return PT_ERR_DATA;
            uint8_t counts[17] = { 0 };
            int total = 0;
            for (int l = 1; l <= 16; l++) { const int v = u8(); if (v < 0) return PT_ERR_DATA; counts[l] = (uint8_t)v; total += v; }
            if (total > 256 || len < 17 + total) return PT_ERR_DATA;
            Huff& t = cls ? ac[id] : dc[id];
            for (int i = 0; i < total; i++) t.vals[i] = (uint8_t)u8();
            // DC symbols are magnitude categories: libjpeg-turbo (jpeg_make_d_derived_tbl) rejects any
            // above 15, which would shift by 16 or more bits in bits() / extend()
            if (!cls)
                for (int i = 0; i < total; i++)
                    if (t.vals[i] > 15) return PT_ERR_DATA;
            memset(t.look, 0, sizeof t.look);
            int code = 0, k = 0;
            for (int l = 1; l <= 16; l++) {
                t.valoff[l] = k - code;
                if (code + counts[l] > (1 << l)) return PT_ERR_DATA;   // more codes than the length allows
                if (counts[l]) {
                    for (int i = 0; i < counts[l]; i++, k++, code++)
                        if (l <= 8)
                            for (int f = 0; f < (1 << (8 - l)); f++) t.look[(code << (8 - l)) | f] = (uint16_t)((l << 8) | t.vals[k]);
                    t.maxcode[l] = code - 1;
                } else t.maxcode[l] = -1;
                code <<= 1;
            }
            t.maxcode[17] = 0x7fffffff;
            t.present = true;
            len -= 17 + total;
        }
        return PT_OK;
    }

    int readSof(int marker)
    {
        if (seenSof) return PT_ERR_DATA;
        seenSof = true;
        if (marker == 0xC2) progressive = true;
        else if (marker != 0xC0 && marker != 0xC1) return PT_ERR_UNSUPPORTED;   // lossless / arithmetic / 12-bit
        if (u8() != 8) return PT_ERR_UNSUPPORTED;
        H = u16(); W = u16(); ncomp = u8();
        if (H <= 0 || W <= 0 || (ncomp != 1 && ncomp != 3)) return PT_ERR_UNSUPPORTED;
        if ((long long)W * H > (1ll << 28)) return PT_ERR_UNSUPPORTED;   // 16k x 16k at most
        for (int i = 0; i < ncomp; i++) {
            c[i].id = u8();
            const int hv = u8();
            c[i].h = hv >> 4; c[i].v = hv & 15; c[i].tq = u8();
            if (c[i].h < 1 || c[i].h > 4 || c[i].v < 1 || c[i].v > 4 || c[i].tq < 0 || c[i].tq > 3) return PT_ERR_DATA;
            hmax = c[i].h > hmax ? c[i].h : hmax;
            vmax = c[i].v > vmax ? c[i].v : vmax;
        }
        mcux = (W + 8 * hmax - 1) / (8 * hmax);
        mcuy = (H + 8 * vmax - 1) / (8 * vmax);
        for (int i = 0; i < ncomp; i++) {
            Comp& k = c[i];
            k.dw = (W * k.h + hmax - 1) / hmax;
            k.dh = (H * k.v + vmax - 1) / vmax;
            k.bw = (k.dw + 7) / 8; k.bh = (k.dh + 7) / 8;
            k.bwm = mcux * k.h; k.bhm = mcuy * k.v;
            k.coef.assign((size_t)k.bwm * k.bhm * 64, 0);
        }
        return PT_OK;
    }

    int16_t* block(Comp& k, int bx, int by) { return &k.coef[((size_t)by * k.bwm + bx) * 64]; }

    void decodeBlockBaseline(Comp& k, int16_t* b)
    {
        const int s = decode(dc[k.td]);
        const int diff = s ? extend(bits(s), s) : 0;
        k.dcpred += diff;
        b[0] = (int16_t)k.dcpred;
        for (int i = 1; i < 64; i++) {
            const int rs = decode(ac[k.ta]);
            const int r = rs >> 4, sz = rs & 15;
            if (sz) { i += r; b[kZigzag[i]] = (int16_t)extend(bits(sz), sz); }
            else { if (r != 15) break; i += 15; }
        }
    }
    // progressive scans (G.1.2): jdphuff.c decode_mcu_DC_first / _DC_refine / _AC_first / _AC_refine
    void dcFirst(Comp& k, int16_t* b, int al)
    {
        const int s = decode(dc[k.td]);
        const int diff = s ? extend(bits(s), s) : 0;
        k.dcpred += diff;
        b[0] = (int16_t)(k.dcpred * (1 << al));
    }
    void dcRefine(int16_t* b, int al) { if (bit()) b[0] = (int16_t)(b[0] | (1 << al)); }
    void acFirst(Comp& k, int16_t* b, int ss, int se, int al)
    {
        if (eobrun > 0) { eobrun--; return; }
        for (int i = ss; i <= se; i++) {
            const int rs = decode(ac[k.ta]);
            const int r = rs >> 4, s = rs & 15;
            if (s) { i += r; b[kZigzag[i]] = (int16_t)(extend(bits(s), s) * (1 << al)); }
            else if (r == 15) i += 15;
            else { eobrun = (1 << r) + (r ? bits(r) : 0) - 1; break; }
        }
    }
    void refineCoef(int16_t* cf, int p1, int m1)
    {
        if (bit() && (*cf & p1) == 0) *cf = (int16_t)(*cf >= 0 ? *cf + p1 : *cf + m1);
    }
    void acRefine(Comp& k, int16_t* b, int ss, int se, int al)
    {
        const int p1 = 1 << al, m1 = (int)((-1u) << al);
        int i = ss;
        if (eobrun == 0) {
            for (; i <= se; i++) {
                const int rs = decode(ac[k.ta]);
                int r = rs >> 4, s = rs & 15;
                if (s) s = bit() ? p1 : m1;
                else if (r != 15) { eobrun = (1 << r) + (r ? bits(r) : 0); break; }
                do {
                    int16_t* cf = &b[kZigzag[i]];
                    if (*cf != 0) refineCoef(cf, p1, m1);
                    else if (--r < 0) break;
                    i++;
                } while (i <= se);
                if (s) b[kZigzag[i]] = (int16_t)s;
            }
        }
        if (eobrun > 0) {
            for (; i <= se; i++) {
                int16_t* cf = &b[kZigzag[i]];
                if (*cf != 0) refineCoef(cf, p1, m1);
            }
            eobrun--;
        }
    }

    // a restart marker after every `restart` MCUs: DC predictions and EOB runs start afresh
    bool restartMarker()
    {
        resetBits();
        while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) p++;
        if (p + 1 >= end) return false;
        p += 2;
        for (int i = 0; i < ncomp; i++) c[i].dcpred = 0;
        eobrun = 0;
        return true;
    }

    int readScan(int len)
    {
        const int ns = u8();
        if (ns < 1 || ns > ncomp || len != 4 + 2 * ns) return PT_ERR_DATA;
        Comp* sc[4];
        for (int i = 0; i < ns; i++) {
            const int id = u8(), t = u8();
            sc[i] = nullptr;
            for (int j = 0; j < ncomp; j++) if (c[j].id == id) sc[i] = &c[j];
            if (!sc[i]) return PT_ERR_DATA;
            sc[i]->td = t >> 4; sc[i]->ta = t & 15;
            if (sc[i]->td > 3 || sc[i]->ta > 3) return PT_ERR_DATA;
        }
        const int ss = u8(), se = u8(), a = u8();
        const int ah = a >> 4, al = a & 15;
        if (ss < 0 || se > 63 || ss > se) return PT_ERR_DATA;
        const bool isDc = ss == 0;
        for (int i = 0; i < ns; i++) {
            if ((!progressive || (isDc && ah == 0)) && !dc[sc[i]->td].present) return PT_ERR_DATA;
            if ((!progressive || !isDc) && !ac[sc[i]->ta].present) return PT_ERR_DATA;
            sc[i]->dcpred = 0;
        }
        resetBits();
        eobrun = 0;
        auto unit = [&](Comp& k, int16_t* b) {
            if (!progressive) decodeBlockBaseline(k, b);
            else if (isDc) { if (ah == 0) dcFirst(k, b, al); else dcRefine(b, al); }
            else if (ah == 0) acFirst(k, b, ss, se, al);
            else acRefine(k, b, ss, se, al);
        };
        int mcus = 0;
        if (ns == 1) {   // non-interleaved: the component's own blocks, raster order
            Comp& k = *sc[0];
            for (int by = 0; by < k.bh; by++)
                for (int bx = 0; bx < k.bw; bx++) {
                    if (restart && mcus && mcus % restart == 0 && !restartMarker()) return PT_ERR_DATA;
                    unit(k, block(k, bx, by));
                    mcus++;
                }
        } else {
            for (int my = 0; my < mcuy; my++)
                for (int mx = 0; mx < mcux; mx++) {
                    if (restart && mcus && mcus % restart == 0 && !restartMarker()) return PT_ERR_DATA;
                    for (int i = 0; i < ns; i++) {
                        Comp& k = *sc[i];
                        for (int y = 0; y < k.v; y++)
                            for (int x = 0; x < k.h; x++) unit(k, block(k, mx * k.h + x, my * k.v + y));
                    }
                    mcus++;
                }
        }
        // skip to the next marker (the bit reader stops in front of it)
        while (p + 1 < end && !(p[0] == 0xFF && p[1] != 0x00 && !(p[1] >= 0xD0 && p[1] <= 0xD7))) p++;
        return PT_OK;
    }

    int parse()
    {
        if (u8() != 0xFF || u8() != 0xD8) return PT_ERR_DATA;
        for (;;) {
            int b;
            do b = u8(); while (b >= 0 && b != 0xFF);   // bytes between segments are skipped
            while (b == 0xFF) b = u8();                  // fill bytes
            if (b < 0) return PT_ERR_DATA;
            const int marker = b;
            if (marker == 0xD9) break;                              // EOI
            if (marker >= 0xD0 && marker <= 0xD7) continue;
            const int len = u16();
            if (len < 2 || p + (len - 2) > end) return PT_ERR_DATA;
            const uint8_t* next = p + (len - 2);
            int rc = PT_OK;
            if (marker == 0xC4) rc = readHuff(len - 2);
            else if (marker == 0xDB) {
                int n = len - 2;
                while (n > 0) {
                    if (n < 65) return PT_ERR_DATA;   // a table cut short by its segment
                    const int pq = u8();
                    if ((pq >> 4) != 0 || (pq & 15) > 3) return PT_ERR_UNSUPPORTED;   // 16-bit tables
                    for (int i = 0; i < 64; i++) q[pq & 15][kZigzag[i]] = (uint16_t)u8();
                    qset[pq & 15] = true;
                    n -= 65;
                }
            } else if (marker == 0xDD) restart = u16();
            else if (marker >= 0xC0 && marker <= 0xCF && marker != 0xC4 && marker != 0xC8 && marker != 0xCC) rc = readSof(marker);
            else if (marker == 0xDA) {
                if (!seenSof) return PT_ERR_DATA;
                rc = readScan(len - 2);
                if (rc != PT_OK) return rc;
                continue;   // p is at the next marker
            } else if (marker == 0xEE && len >= 14) {   // Adobe: transform byte at offset 11
                adobe = true;
                adobeTransform = p[11];
            }
            if (rc != PT_OK) return rc;
            p = next;
        }
        if (!seenSof) return PT_ERR_DATA;
        if (ncomp == 3 && adobe && adobeTransform == 0) return PT_ERR_UNSUPPORTED;   // stored RGB
        return PT_OK;
    }
};

// jidctint.c jpeg_idct_islow (8-bit samples) with the post-IDCT range-limit table of jdmaster.c
constexpr int kConstBits = 13, kPass1Bits = 2;
inline int64_t mul(int64_t v, int64_t c) { return v * c; }
inline int64_t descale(int64_t x, int n) { return (x + ((int64_t)1 << (n - 1))) >> n; }

struct RangeLimit {
    uint8_t t[1024];   // idct_range_limit[x & 1023]
    RangeLimit()
    {
        for (int j = 0; j < 1024; j++)
            t[j] = j < 128 ? (uint8_t)(j + 128) : j < 512 ? 255 : j < 896 ? 0 : (uint8_t)(j - 896);
    }
};

void idctIslow(const int16_t* in, const uint16_t* qt, uint8_t* out, int stride, const uint8_t* rl)
{
    int ws[64];
    for (int col = 0; col < 8; col++) {
        const int16_t* ip = in + col;
        const uint16_t* qp = qt + col;
        int* wp = ws + col;
        if (ip[8] == 0 && ip[16] == 0 && ip[24] == 0 && ip[32] == 0 && ip[40] == 0 && ip[48] == 0 && ip[56] == 0) {
            const int dc = (ip[0] * (int)qp[0]) * (1 << kPass1Bits);
            for (int r = 0; r < 8; r++) wp[8 * r] = dc;
            continue;
        }
        int64_t z2 = ip[16] * (int64_t)qp[16], z3 = ip[48] * (int64_t)qp[48];
        int64_t z1 = mul(z2 + z3, 4433);
        int64_t tmp2 = z1 + mul(z3, -15137), tmp3 = z1 + mul(z2, 6270);
        z2 = ip[0] * (int64_t)qp[0]; z3 = ip[32] * (int64_t)qp[32];
        int64_t tmp0 = (z2 + z3) * (1 << kConstBits), tmp1 = (z2 - z3) * (1 << kConstBits);
        const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = ip[56] * (int64_t)qp[56]; tmp1 = ip[40] * (int64_t)qp[40];
        tmp2 = ip[24] * (int64_t)qp[24]; tmp3 = ip[8] * (int64_t)qp[8];
        z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        const int64_t z5 = mul(z3 + z4, 9633);
        tmp0 = mul(tmp0, 2446); tmp1 = mul(tmp1, 16819); tmp2 = mul(tmp2, 25172); tmp3 = mul(tmp3, 12299);
        z1 = mul(z1, -7373); z2 = mul(z2, -20995); z3 = mul(z3, -16069); z4 = mul(z4, -3196);
        z3 += z5; z4 += z5;
        tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
        const int sh = kConstBits - kPass1Bits;
        wp[0] = (int)descale(tmp10 + tmp3, sh);  wp[56] = (int)descale(tmp10 - tmp3, sh);
        wp[8] = (int)descale(tmp11 + tmp2, sh);  wp[48] = (int)descale(tmp11 - tmp2, sh);
        wp[16] = (int)descale(tmp12 + tmp1, sh); wp[40] = (int)descale(tmp12 - tmp1, sh);
        wp[24] = (int)descale(tmp13 + tmp0, sh); wp[32] = (int)descale(tmp13 - tmp0, sh);
    }
    for (int row = 0; row < 8; row++) {
        const int* wp = ws + 8 * row;
        uint8_t* op = out + (size_t)row * stride;
        const int sh = kConstBits + kPass1Bits + 3;
        if (wp[1] == 0 && wp[2] == 0 && wp[3] == 0 && wp[4] == 0 && wp[5] == 0 && wp[6] == 0 && wp[7] == 0) {
            const uint8_t dc = rl[(int)descale(wp[0], kPass1Bits + 3) & 1023];
            for (int i = 0; i < 8; i++) op[i] = dc;
            continue;
        }
        int64_t z2 = wp[2], z3 = wp[6];
        int64_t z1 = mul(z2 + z3, 4433);
        int64_t tmp2 = z1 + mul(z3, -15137), tmp3 = z1 + mul(z2, 6270);
        int64_t tmp0 = ((int64_t)wp[0] + wp[4]) * (1 << kConstBits), tmp1 = ((int64_t)wp[0] - wp[4]) * (1 << kConstBits);
        const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = wp[7]; tmp1 = wp[5]; tmp2 = wp[3]; tmp3 = wp[1];
        z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        const int64_t z5 = mul(z3 + z4, 9633);
        tmp0 = mul(tmp0, 2446); tmp1 = mul(tmp1, 16819); tmp2 = mul(tmp2, 25172); tmp3 = mul(tmp3, 12299);
        z1 = mul(z1, -7373); z2 = mul(z2, -20995); z3 = mul(z3, -16069); z4 = mul(z4, -3196);
        z3 += z5; z4 += z5;
        tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
        op[0] = rl[(int)descale(tmp10 + tmp3, sh) & 1023]; op[7] = rl[(int)descale(tmp10 - tmp3, sh) & 1023];
        op[1] = rl[(int)descale(tmp11 + tmp2, sh) & 1023]; op[6] = rl[(int)descale(tmp11 - tmp2, sh) & 1023];
        op[2] = rl[(int)descale(tmp12 + tmp1, sh) & 1023]; op[5] = rl[(int)descale(tmp12 - tmp1, sh) & 1023];
        op[3] = rl[(int)descale(tmp13 + tmp0, sh) & 1023]; op[4] = rl[(int)descale(tmp13 - tmp0, sh) & 1023];
    }
}

// the component plane upsampled to the image grid (jdsample.c; context rows replicate the edges)
int upsample(const Comp& k, int hmax, int vmax, const uint8_t* in, int istride, int W, int H, std::vector<uint8_t>& out)
{
    out.assign((size_t)W * H, 0);
    const int fh = hmax / k.h, fv = vmax / k.v;
    if (hmax % k.h || vmax % k.v) return PT_ERR_UNSUPPORTED;
    auto row = [&](int r) { r = r < 0 ? 0 : r >= k.dh ? k.dh - 1 : r; return in + (size_t)r * istride; };
    std::vector<uint8_t> line((size_t)k.dw * 2 + 2);
    for (int y = 0; y < H; y++) {
        const uint8_t* src;
        if (fv == 1) src = row(y);
        else if (fv == 2) {   // vertical triangle filter rows (h1v2 alone; h2v2 below does both)
            if (fh == 1) {
                const int r = y >> 1, vsub = y & 1;
                const uint8_t* i0 = row(r);
                const uint8_t* i1 = row(vsub ? r + 1 : r - 1);
                const int bias = vsub ? 2 : 1;
                for (int x = 0; x < k.dw; x++) line[x] = (uint8_t)((i0[x] * 3 + i1[x] + bias) >> 2);
                src = line.data();
            } else src = nullptr;
        } else return PT_ERR_UNSUPPORTED;
        uint8_t* o = out.data() + (size_t)y * W;
        if (fh == 1 && fv <= 2 && src) { memcpy(o, src, (size_t)W); continue; }
        if (fh == 2 && fv == 1) {   // h2v1_fancy_upsample
            const uint8_t* ip = src;
            const int dw = k.dw;
            if (dw <= 2) { for (int x = 0; x < W; x++) o[x] = ip[x >> 1]; continue; }
            uint8_t* t = line.data();
            int n = 0;
            t[n++] = ip[0];
            t[n++] = (uint8_t)((ip[0] * 3 + ip[1] + 2) >> 2);
            for (int x = 1; x < dw - 1; x++) {
                const int v3 = ip[x] * 3;
                t[n++] = (uint8_t)((v3 + ip[x - 1] + 1) >> 2);
                t[n++] = (uint8_t)((v3 + ip[x + 1] + 2) >> 2);
            }
            t[n++] = (uint8_t)((ip[dw - 1] * 3 + ip[dw - 2] + 1) >> 2);
            t[n++] = ip[dw - 1];
            memcpy(o, t, (size_t)W);
            continue;
        }
        if (fh == 2 && fv == 2) {   // h2v2_fancy_upsample
            const int r = y >> 1, vsub = y & 1;
            const uint8_t* i0 = row(r);
            const uint8_t* i1 = row(vsub ? r + 1 : r - 1);
            const int dw = k.dw;
            if (dw <= 2) { for (int x = 0; x < W; x++) o[x] = i0[x >> 1]; continue; }   // h2v2_upsample (box)
            uint8_t* t = line.data();
            int n = 0;
            int thiscol = i0[0] * 3 + i1[0], nextcol = i0[1] * 3 + i1[1], lastcol;
            t[n++] = (uint8_t)((thiscol * 4 + 8) >> 4);
            t[n++] = (uint8_t)((thiscol * 3 + nextcol + 7) >> 4);
            lastcol = thiscol; thiscol = nextcol;
            for (int x = 2; x < dw; x++) {
                nextcol = i0[x] * 3 + i1[x];
                t[n++] = (uint8_t)((thiscol * 3 + lastcol + 8) >> 4);
                t[n++] = (uint8_t)((thiscol * 3 + nextcol + 7) >> 4);
                lastcol = thiscol; thiscol = nextcol;
            }
            t[n++] = (uint8_t)((thiscol * 3 + lastcol + 8) >> 4);
            t[n++] = (uint8_t)((thiscol * 4 + 7) >> 4);
            memcpy(o, t, (size_t)W);
            continue;
        }
        return PT_ERR_UNSUPPORTED;
    }
    return PT_OK;
}

int decodeJpeg(const uint8_t* data, size_t size, int* w, int* h, uint8_t* rgba, size_t cap, bool infoOnly)
{
    if (!data || size < 4) return PT_ERR_ARG;
    Decoder d;
    d.p = data; d.end = data + size;
    if (infoOnly) {   // dimensions from the frame header only
        const uint8_t* q = data + 2;
        while (q + 9 < d.end) {
            if (q[0] != 0xFF) { q++; continue; }
            const int m = q[1];
            if (m == 0xFF) { q++; continue; }
            if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) { q += 2; continue; }
            const int len = (q[2] << 8) | q[3];
            if (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
                *h = (q[5] << 8) | q[6]; *w = (q[7] << 8) | q[8];
                return PT_OK;
            }
            q += 2 + len;
        }
        return PT_ERR_DATA;
    }
    int rc = d.parse();
    if (rc != PT_OK) return rc;
    for (int i = 0; i < d.ncomp; i++)   // libjpeg-turbo: JERR_NO_QUANT_TABLE
        if (!d.qset[d.c[i].tq]) return PT_ERR_DATA;
    *w = d.W; *h = d.H;
    if (!rgba) return PT_OK;
    if (cap < (size_t)d.W * d.H * 4) return PT_ERR_ARG;
    static const RangeLimit rlim;
    std::vector<uint8_t> plane[3];
    for (int i = 0; i < d.ncomp; i++) {
        Comp& k = d.c[i];
        const int pw = k.bw * 8, ph = k.bh * 8;
        std::vector<uint8_t> samp((size_t)pw * ph);
        for (int by = 0; by < k.bh; by++)
            for (int bx = 0; bx < k.bw; bx++)
                idctIslow(d.block(k, bx, by), d.q[k.tq], samp.data() + (size_t)by * 8 * pw + bx * 8, pw, rlim.t);
        rc = upsample(k, d.hmax, d.vmax, samp.data(), pw, d.W, d.H, plane[i]);
        if (rc != PT_OK) return rc;
    }
    const size_t n = (size_t)d.W * d.H;
    if (d.ncomp == 1) {
        for (size_t j = 0; j < n; j++) { const uint8_t g = plane[0][j]; rgba[4 * j] = rgba[4 * j + 1] = rgba[4 * j + 2] = g; rgba[4 * j + 3] = 255; }
        return PT_OK;
    }
    // jdcolor.c build_ycc_rgb_table / ycc_rgb_convert: SCALEBITS 16, FIX(x) = x * 65536 + 0.5
    int crr[256], cbb[256], crg[256], cbg[256];
    for (int i = 0; i < 256; i++) {
        const int64_t x = i - 128;
        crr[i] = (int)((91881 * x + 32768) >> 16);
        cbb[i] = (int)((116130 * x + 32768) >> 16);
        crg[i] = (int)(-46802 * x);
        cbg[i] = (int)(-22554 * x + 32768);
    }
    auto clamp = [](int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); };
    for (size_t j = 0; j < n; j++) {
        const int y = plane[0][j], cb = plane[1][j], cr = plane[2][j];
        rgba[4 * j] = clamp(y + crr[cr]);
        rgba[4 * j + 1] = clamp(y + ((cbg[cb] + crg[cr]) >> 16));
        rgba[4 * j + 2] = clamp(y + cbb[cb]);
        rgba[4 * j + 3] = 255;
    }
    return PT_OK;
}

}  // namespace

extern "C" int pt_jpeg_size(const uint8_t* data, size_t size, int* width, int* height)
{
    if (!width || !height) return PT_ERR_ARG;
    return decodeJpeg(data, size, width, height, nullptr, 0, true);
}

extern "C" int pt_jpeg_decode_rgba8(const uint8_t* data, size_t size, uint8_t* rgba, size_t capacity)
{
    int w = 0, h = 0;
    if (!rgba) return PT_ERR_ARG;
    try {
        return decodeJpeg(data, size, &w, &h, rgba, capacity, false);
    } catch (const std::bad_alloc&) {
        return PT_ERR_OOM;
    }
}
