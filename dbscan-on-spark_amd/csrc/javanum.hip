// javanum.hip -- host code: the JVM number semantics the reference's driver and text output
// depend on, restated exactly (Spark 2.1.0 / Scala 2.10 run on JDK 7/8, pom.xml:30-37).
//
//   jdk8_double_string   java.lang.Double.toString(double) as JDK 7/8 print it: the digit
//                        generation of sun.misc.FloatingDecimal (BinaryToASCIIBuffer.dtoa): the
//                        integer fast path (|d| < 2^63 with no fraction bits) keeps every digit
//                        above the "insignificant" ones implied by the half-ulp, so e.g.
//                        2.82879384806159E17 prints as 2.82879384806159008E17; the general path
//                        is Steele & White's digit loop with a SYMMETRIC stopping test (the
//                        asymmetric spacing below powers of two is ignored) and at least two
//                        digits in E-form.  JDK >= 19 prints the shortest digits instead.
//   scala_range_count    Scala 2.10 NumericRange.count(start, end, step, isInclusive) for
//                        Double ranges (`a until b by s`, EvenSplitPartitioner.scala:150-152):
//                        the Double difference end - start, then Numeric.DoubleAsIfIntegral's
//                        quot / rem through BigDecimal(Double.toString(_)) at DECIMAL128 (34
//                        digits, HALF_EVEN), the quotient's doubleValue truncated toLong.
//
// Arbitrary-precision unsigned integers below are plain schoolbook limbs: exact, not fast; the
// big path of dtoa runs only for values outside the integer fast path and the long/int paths.
#include "internal.h"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace dbscan {
namespace {

struct Big {  // unsigned, little-endian 32-bit limbs, no leading zero limbs
    std::vector<uint32_t> w;
    Big() = default;
    explicit Big(uint64_t v) {
        while (v) {
            w.push_back((uint32_t)v);
            v >>= 32;
        }
    }
    bool zero() const { return w.empty(); }
    void trim() {
        while (!w.empty() && w.back() == 0) w.pop_back();
    }
    Big& mul_small(uint32_t m) {
        uint64_t c = 0;
        for (uint32_t& x : w) {
            const uint64_t t = (uint64_t)x * m + c;
            x = (uint32_t)t;
            c = t >> 32;
        }
        if (c) w.push_back((uint32_t)c);
        trim();
        return *this;
    }
    Big& mul_pow5(int k) {
        for (; k >= 13; k -= 13) mul_small(1220703125u);  // 5^13
        uint32_t p = 1;
        while (k-- > 0) p *= 5;
        return mul_small(p);
    }
    Big& mul_pow10(int k) {
        mul_pow5(k);
        return shl(k);
    }
    Big& shl(int bits) {
        if (zero() || bits == 0) return *this;
        const int limbs = bits / 32, b = bits % 32;
        std::vector<uint32_t> r((size_t)limbs, 0u);
        uint32_t carry = 0;
        for (uint32_t x : w) {
            r.push_back(b ? (x << b) | carry : x);
            carry = b ? x >> (32 - b) : 0;
        }
        if (carry) r.push_back(carry);
        w.swap(r);
        trim();
        return *this;
    }
    static int cmp(const Big& a, const Big& b) {
        if (a.w.size() != b.w.size()) return a.w.size() < b.w.size() ? -1 : 1;
        for (size_t i = a.w.size(); i-- > 0;)
            if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
        return 0;
    }
    static Big add(const Big& a, const Big& b) {
        Big r;
        const size_t n = std::max(a.w.size(), b.w.size());
        uint64_t c = 0;
        for (size_t i = 0; i < n; ++i) {
            const uint64_t t = c + (i < a.w.size() ? a.w[i] : 0u) + (i < b.w.size() ? b.w[i] : 0u);
            r.w.push_back((uint32_t)t);
            c = t >> 32;
        }
        if (c) r.w.push_back((uint32_t)c);
        r.trim();
        return r;
    }
    Big& sub(const Big& b) {  // requires *this >= b
        int64_t br = 0;
        for (size_t i = 0; i < w.size(); ++i) {
            int64_t t = (int64_t)w[i] - br - (i < b.w.size() ? (int64_t)b.w[i] : 0);
            br = t < 0;
            if (t < 0) t += (int64_t)1 << 32;
            w[i] = (uint32_t)t;
        }
        trim();
        return *this;
    }
    // q = floor(*this / d) for a quotient known to be small; *this becomes the remainder
    int64_t divmod_small_quotient(const Big& d) {
        int64_t q = 0;
        while (cmp(*this, d) >= 0) {
            sub(d);
            ++q;
        }
        return q;
    }
    // long division: *this = floor(*this / d), returns the remainder (general sizes)
    Big divmod(const Big& d) {
        Big q, r;
        const size_t nbits = w.size() * 32;
        for (size_t i = nbits; i-- > 0;) {
            r.shl(1);
            if ((w[i / 32] >> (i % 32)) & 1u) {
                if (r.w.empty()) r.w.push_back(0);
                r.w[0] |= 1u;
            }
            if (cmp(r, d) >= 0) {
                r.sub(d);
                if (q.w.size() < i / 32 + 1) q.w.resize(i / 32 + 1, 0u);
                q.w[i / 32] |= 1u << (i % 32);
            }
        }
        q.trim();
        w.swap(q.w);
        return r;
    }
    bool odd() const { return !w.empty() && (w[0] & 1u); }
    std::string decimal() const {
        if (zero()) return "0";
        Big t = *this;
        std::string s;
        while (!t.zero()) {
            uint64_t rem = 0;
            for (size_t i = t.w.size(); i-- > 0;) {
                const uint64_t cur = (rem << 32) | t.w[i];
                t.w[i] = (uint32_t)(cur / 1000000000u);
                rem = cur % 1000000000u;
            }
            t.trim();
            char buf[16];
            snprintf(buf, sizeof buf, t.zero() ? "%llu" : "%09llu", (unsigned long long)rem);
            s.insert(0, buf);
        }
        return s;
    }
};

// ------------------------------ FloatingDecimal (JDK 7/8) --------------------------------
constexpr int kExpShift = 52;
constexpr uint64_t kFractHob = 1ull << 52;
constexpr int kMaxSmallBinExp = 62;
constexpr int kMinSmallBinExp = -(63 / 3);

int n5bits(int k) {  // bits of 5^k (FloatingDecimal.N_5_BITS), k >= 0
    if (k == 0) return 0;
    return (int)std::floor(k * 2.321928094887362) + 1;
}

uint64_t pow5_u64(int k) {
    uint64_t p = 1;
    while (k-- > 0) p *= 5;
    return p;
}

// floor(log10(2^p2)) for 2 <= p2 (FloatingDecimal.insignificantDigitsForPow2), else 0
int insignificant_digits_pow2(int p2) {
    if (p2 <= 1 || p2 >= 64) return 0;
    const uint64_t v = 1ull << p2;
    int i = 0;
    for (uint64_t t = v; t >= 10; t /= 10) ++i;
    return i;
}

int estimate_dec_exp(uint64_t fract_bits, int bin_exp) {
#pragma clang fp contract(off)
    uint64_t b = 0x3FF0000000000000ull | (fract_bits & 0x000FFFFFFFFFFFFFull);
    double d2;
    memcpy(&d2, &b, 8);
    const double d = (d2 - 1.5) * 0.289529654 + 0.176091259 + (double)bin_exp * 0.301029995663981;
    return (int)std::floor(d);  // FloatingDecimal.estimateDecExp: floor, computed on the bits
}

struct Digits {
    char d[32];
    int n = 0;
    int dec_exp = 0;  // value = 0.d1d2... x 10^dec_exp
};

void roundup(Digits& g) {
    int i = g.n - 1;
    char q = g.d[i];
    if (q == '9') {
        while (q == '9' && i > 0) {
            g.d[i] = '0';
            q = g.d[--i];
        }
        if (q == '9') {
            g.dec_exp += 1;
            g.d[0] = '1';
            return;
        }
    }
    g.d[i] = (char)(q + 1);
}

void develop_long_digits(Digits& g, int dec_exp, uint64_t lvalue, int insignificant) {
    if (insignificant != 0) {
        const uint64_t pow10 = pow5_u64(insignificant) << insignificant;
        const uint64_t residue = lvalue % pow10;
        lvalue /= pow10;
        dec_exp += insignificant;
        if (residue >= (pow10 >> 1)) lvalue++;
    }
    char tmp[32];
    int pos = 31;
    int c = (int)(lvalue % 10);
    lvalue /= 10;
    while (c == 0) {
        dec_exp++;
        c = (int)(lvalue % 10);
        lvalue /= 10;
    }
    while (lvalue != 0) {
        tmp[pos--] = (char)('0' + c);
        dec_exp++;
        c = (int)(lvalue % 10);
        lvalue /= 10;
    }
    tmp[pos] = (char)('0' + c);
    g.n = 32 - pos;
    memcpy(g.d, tmp + pos, (size_t)g.n);
    g.dec_exp = dec_exp + 1;
}

// BinaryToASCIIBuffer.dtoa(binExp, fractBits, nSignificantBits, isCompatibleFormat = true)
void dtoa(Digits& g, int bin_exp, uint64_t fract_bits, int n_significant_bits) {
    const int tail_zeros = __builtin_ctzll(fract_bits);
    const int n_fract_bits = kExpShift + 1 - tail_zeros;
    const int n_tiny_bits = std::max(0, n_fract_bits - bin_exp - 1);
    if (bin_exp <= kMaxSmallBinExp && bin_exp >= kMinSmallBinExp) {
        if (n_tiny_bits < 27 && n_fract_bits + n5bits(n_tiny_bits) < 64 && n_tiny_bits == 0) {
            const int insignificant =
                bin_exp > n_significant_bits
                    ? insignificant_digits_pow2(bin_exp - n_significant_bits - 1)
                    : 0;
            uint64_t fb = fract_bits;
            if (bin_exp >= kExpShift)
                fb <<= (bin_exp - kExpShift);
            else
                fb >>= (kExpShift - bin_exp);
            develop_long_digits(g, 0, fb, insignificant);
            return;
        }
    }
    int dec_exp = estimate_dec_exp(fract_bits, bin_exp);
    int B5 = std::max(0, -dec_exp);
    int B2 = B5 + n_tiny_bits + bin_exp;
    int S5 = std::max(0, dec_exp);
    int S2 = S5 + n_tiny_bits;
    int M5 = B5;
    int M2 = B2 - n_significant_bits;
    uint64_t fb = fract_bits >> tail_zeros;
    B2 -= n_fract_bits - 1;
    const int common2 = std::min(B2, S2);
    B2 -= common2;
    S2 -= common2;
    M2 -= common2;
    if (n_fract_bits == 1) M2 -= 1;  // (the JDK's power-of-two "HACK")
    if (M2 < 0) {
        B2 -= M2;
        S2 -= M2;
        M2 = 0;
    }
    int ndigit = 0;
    bool low, high;
    int64_t low_digit_difference = 0;
    const int b_bits = n_fract_bits + B2 + (B5 < 27 ? n5bits(B5) : B5 * 3);
    const int ten_s_bits = S2 + 1 + (S5 + 1 < 27 ? n5bits(S5 + 1) : (S5 + 1) * 3);
    if (b_bits < 64 && ten_s_bits < 64) {
        // the int and long paths of the JDK: the same arithmetic (the values fit in 64 bits)
        int64_t b = (int64_t)((fb * pow5_u64(B5)) << B2);
        const int64_t s = (int64_t)(pow5_u64(S5) << S2);
        int64_t m = (int64_t)(pow5_u64(M5) << M2);
        const int64_t tens = s * 10;
        const bool is_int = b_bits < 32 && ten_s_bits < 32;
        // Java int (long) arithmetic wraps: b + m and 2b - tens as the JDK's int / long paths
        const auto wrap = [&](uint64_t v) -> int64_t {
            return is_int ? (int64_t)(int32_t)(uint32_t)v : (int64_t)v;
        };
        int q = (int)(b / s);
        b = 10 * (b % s);
        m = wrap((uint64_t)m * 10u);
        low = b < m;
        high = wrap((uint64_t)b + (uint64_t)m) > tens;
        if (q == 0 && !high)
            dec_exp--;
        else
            g.d[ndigit++] = (char)('0' + q);
        if (dec_exp < -3 || dec_exp >= 8) high = low = false;
        while (!low && !high) {
            q = (int)(b / s);
            b = 10 * (b % s);
            m = wrap((uint64_t)m * 10u);
            if (m > 0) {
                low = b < m;
                high = wrap((uint64_t)b + (uint64_t)m) > tens;
            } else {
                low = true;
                high = true;
            }
            g.d[ndigit++] = (char)('0' + q);
        }
        low_digit_difference = wrap(((uint64_t)b << 1) - (uint64_t)tens);
    } else {
        Big Sv = Big(1).mul_pow5(S5).shl(S2);
        Big Bv = Big(fb).mul_pow5(B5).shl(B2);
        Big Mv = Big(1).mul_pow5(M5 + 1).shl(M2 + 1);
        Big tenS = Big(1).mul_pow5(S5 + 1).shl(S2 + 1);
        const auto quo_rem = [&]() {  // q = B / S; B = 10 * (B % S)
            const int q = (int)Bv.divmod_small_quotient(Sv);
            Bv.mul_small(10);
            return q;
        };
        int q = quo_rem();
        low = Big::cmp(Bv, Mv) < 0;
        high = Big::cmp(tenS, Big::add(Bv, Mv)) <= 0;
        if (q == 0 && !high)
            dec_exp--;
        else
            g.d[ndigit++] = (char)('0' + q);
        if (dec_exp < -3 || dec_exp >= 8) high = low = false;
        while (!low && !high) {
            q = quo_rem();
            Mv.mul_small(10);
            low = Big::cmp(Bv, Mv) < 0;
            high = Big::cmp(tenS, Big::add(Bv, Mv)) <= 0;
            g.d[ndigit++] = (char)('0' + q);
        }
        if (high && low) {
            Big b2 = Bv;
            b2.shl(1);
            low_digit_difference = Big::cmp(b2, tenS);
        } else {
            low_digit_difference = 0;
        }
    }
    g.dec_exp = dec_exp + 1;
    g.n = ndigit;
    if (high) {
        if (low) {
            if (low_digit_difference == 0) {
                if ((g.d[g.n - 1] - '0') & 1) roundup(g);
            } else if (low_digit_difference > 0) {
                roundup(g);
            }
        } else {
            roundup(g);
        }
    }
}

}  // namespace

int jdk8_double_string(double d, char* buf) {
    uint64_t bits;
    memcpy(&bits, &d, 8);
    const bool neg = (bits >> 63) != 0;
    uint64_t fract = bits & 0x000FFFFFFFFFFFFFull;
    int bin_exp = (int)((bits >> 52) & 0x7FF);
    if (bin_exp == 0x7FF) {
        if (fract == 0) return sprintf(buf, neg ? "-Infinity" : "Infinity");
        return sprintf(buf, "NaN");
    }
    int n_sig;
    if (bin_exp == 0) {
        if (fract == 0) return sprintf(buf, neg ? "-0.0" : "0.0");
        const int lz = __builtin_clzll(fract);
        const int shift = lz - (63 - kExpShift);
        fract <<= shift;
        bin_exp = 1 - shift;
        n_sig = 64 - lz;
    } else {
        fract |= kFractHob;
        n_sig = kExpShift + 1;
    }
    bin_exp -= 1023;
    Digits g;
    dtoa(g, bin_exp, fract, n_sig);
    // BinaryToASCIIBuffer.getChars
    char* p = buf;
    if (neg) *p++ = '-';
    const int e10 = g.dec_exp;
    if (e10 > 0 && e10 < 8) {
        int len = std::min(g.n, e10);
        memcpy(p, g.d, (size_t)len);
        p += len;
        if (len < e10) {
            for (int i = 0; i < e10 - len; ++i) *p++ = '0';
            *p++ = '.';
            *p++ = '0';
        } else {
            *p++ = '.';
            if (len < g.n) {
                memcpy(p, g.d + len, (size_t)(g.n - len));
                p += g.n - len;
            } else {
                *p++ = '0';
            }
        }
    } else if (e10 <= 0 && e10 > -3) {
        *p++ = '0';
        *p++ = '.';
        for (int i = 0; i < -e10; ++i) *p++ = '0';
        memcpy(p, g.d, (size_t)g.n);
        p += g.n;
    } else {
        *p++ = g.d[0];
        *p++ = '.';
        if (g.n > 1) {
            memcpy(p, g.d + 1, (size_t)(g.n - 1));
            p += g.n - 1;
        } else {
            *p++ = '0';
        }
        *p++ = 'E';
        int e;
        if (e10 <= 0) {
            *p++ = '-';
            e = -e10 + 1;
        } else {
            e = e10 - 1;
        }
        p += sprintf(p, "%d", e);
    }
    *p = 0;
    return (int)(p - buf);
}

namespace {
// The decimal value of Double.toString(d) (JDK 7/8) as (digits, exponent): |d| = D x 10^e.
void java_decimal(double d, Big* D, int* e, bool* neg) {
    char s[64];
    jdk8_double_string(d, s);
    const char* p = s;
    *neg = *p == '-';
    if (*neg) ++p;
    std::string digits;
    int frac = 0, exp10 = 0;
    bool dot = false;
    for (; *p && *p != 'E'; ++p) {
        if (*p == '.') {
            dot = true;
            continue;
        }
        digits.push_back(*p);
        if (dot) ++frac;
    }
    if (*p == 'E') exp10 = atoi(p + 1);
    Big v;
    for (char c : digits) v.mul_small(10), v = Big::add(v, Big((uint64_t)(c - '0')));
    *D = v;
    *e = exp10 - frac;
}
}  // namespace

int64_t scala_range_count(double start, double end, double step, bool inclusive) {
    if (step == 0.0) throw ArgError{"NumericRange: step cannot be 0."};
    if (start == end) return inclusive ? 1 : 0;
    const bool upward = start < end, pos_step = step > 0.0;
    if (upward != pos_step) return 0;
    const double diff = end - start;  // Numeric.DoubleIsConflicted.minus (Double arithmetic)
    // BigDecimal(Double.toString(v)) throws NumberFormatException for "Infinity" / "NaN"
    if (!std::isfinite(diff) || !std::isfinite(step))
        throw ArgError{"NumericRange: BigDecimal of a non-finite Double (NumberFormatException)"};
    Big D, S;
    int a, b;
    bool nd, ns;
    java_decimal(diff, &D, &a, &nd);
    java_decimal(step, &S, &b, &ns);
    if (D.zero()) return inclusive ? 1 : 0;  // (diff rounded to 0 only for denormal gaps)
    // rem == 0 <=> the decimal diff is an exact multiple of the decimal step
    bool exact;
    {
        Big num = D, den = S;
        if (a >= b) num.mul_pow10(a - b); else den.mul_pow10(b - a);
        exact = num.divmod(den).zero();
    }
    // quot: the exact decimal quotient rounded to 34 significant digits (HALF_EVEN), then its
    // doubleValue (Double.parseDouble of the decimal: correctly rounded) truncated toLong
    const int dD = (int)D.decimal().size(), dS = (int)S.decimal().size();
    int t = 34 - (dD - dS + a - b) + 1;  // scale so the integer quotient has >= 34 digits
    Big qv, rem, den;
    for (int iter = 0; iter < 3; ++iter) {
        Big num = D;
        den = S;
        const int ex = a - b + t;  // quotient x 10^t = D x 10^(a-b+t) / S
        if (ex >= 0) num.mul_pow10(ex); else den.mul_pow10(-ex);
        rem = num.divmod(den);
        qv = num;
        const int nq = (int)qv.decimal().size();
        if (nq > 34) {  // drop the extra digits, keep the remainder exact for the rounding
            t -= nq - 34;
            continue;
        }
        break;
    }
    // HALF_EVEN on the remainder
    Big twice = rem;
    twice.shl(1);
    const int c = Big::cmp(twice, den);
    if (c > 0 || (c == 0 && qv.odd())) qv = Big::add(qv, Big(1));
    const std::string s = qv.decimal() + "e" + std::to_string(-t);
    const double qd = strtod(s.c_str(), nullptr);
    // Double.toLong truncates; any count past Int.MaxValue throws in the reference (Java's
    // long overflow of jumps + 1 included), so check before adding
    if (!(qd < 2147483648.0))
        throw ArgError{"NumericRange: seqs cannot contain more than Int.MaxValue elements."};
    const int64_t jumps = qd > 0 ? (int64_t)qd : 0;
    const int64_t count = jumps + ((!inclusive && exact) ? 0 : 1);
    if (count > INT32_MAX)
        throw ArgError{"NumericRange: seqs cannot contain more than Int.MaxValue elements."};
    return count;
}

}  // namespace dbscan
