"""JVM / Scala 2.10 number semantics the reference's partitioner depends on, restated in Python
for the ORACLE (test infrastructure only: nothing in the product imports this module).

The reference runs on Scala 2.10.4 (pom.xml:33-34) and Spark 2.1.0 on a JDK 7/8 runtime.  Two
places of its partitioner reach below the Scala source into the platform:

  * EvenSplitPartitioner.scala:150-152 `(box.x + mrs) until box.x2 by mrs` -- a Double
    NumericRange whose length goes through BigDecimal(Double.toString(d)); Double.toString is
    sun.misc.FloatingDecimal's digit generation as JDK 7/8 print it (restated here as
    `jdk8_double_string`, independently of the product's csrc/javanum.hip);
  * EvenSplitPartitioner.scala:105-123,148-162 `split` reduces over `splits.toSet`: the first
    minimum-cost candidate in the Set's iteration order wins.  Scala 2.10's immutable Set keeps
    insertion order up to 4 elements (Set1..Set4) and above that is a HashTrieSet ordered by the
    "improved" hash of each element, whose hashCode is the case class's MurmurHash3.productHash
    over its four Double fields, each hashed by BoxesRunTime.hashFromDouble (restated here as
    `split_order_key`, independently of the product's csrc/partition.hip).

Only the arithmetic is restated; the algorithms are the published ones of the Scala 2.10.4
library (scala.util.hashing.MurmurHash3, scala.collection.immutable.HashSet,
scala.runtime.BoxesRunTime) and the JDK 8 sun.misc.FloatingDecimal.BinaryToASCIIBuffer.
"""
import struct

_M32 = 0xFFFFFFFF


def _i32(v: int) -> int:
    """Java int wrap-around."""
    v &= _M32
    return v - (1 << 32) if v >> 31 else v


def _i64(v: int) -> int:
    """Java long wrap-around."""
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >> 63 else v


def _bits(d: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", d))[0]


# ------------------------------------------------------------------------------------------
# java.lang.Double.toString (JDK 7/8: sun.misc.FloatingDecimal, BinaryToASCIIBuffer.dtoa)
# ------------------------------------------------------------------------------------------
def _n5bits(k: int) -> int:  # FloatingDecimal.N_5_BITS[k]: bits of 5^k (0 for k = 0)
    return 0 if k == 0 else (5 ** k).bit_length()


def _insignificant_pow2(p2: int) -> int:  # FloatingDecimal.insignificantDigitsForPow2
    return len(str(1 << p2)) - 1 if 1 < p2 < 64 else 0


def _estimate_dec_exp(fract: int, bin_exp: int) -> int:  # FloatingDecimal.estimateDecExp
    d2 = struct.unpack("<d", struct.pack("<Q", 0x3FF0000000000000 | (fract & ((1 << 52) - 1))))[0]
    d = (d2 - 1.5) * 0.289529654 + 0.176091259 + float(bin_exp) * 0.301029995663981
    import math
    return math.floor(d)


def _dtoa(bin_exp: int, fract: int, nsig: int):
    """Returns (digit string, decExponent): value = 0.d1d2... x 10^decExponent."""
    tail = (fract & -fract).bit_length() - 1
    nfract = 53 - tail
    ntiny = max(0, nfract - bin_exp - 1)
    if -21 <= bin_exp <= 62 and ntiny < 27 and nfract + _n5bits(ntiny) < 64 and ntiny == 0:
        # an integer below 2^63: its long value, less the digits below the half ulp
        insig = _insignificant_pow2(bin_exp - nsig - 1) if bin_exp > nsig else 0
        lv = fract << (bin_exp - 52) if bin_exp >= 52 else fract >> (52 - bin_exp)
        dec = 0
        if insig:
            p10 = 10 ** insig
            res = lv % p10
            lv //= p10
            dec += insig
            if res >= p10 >> 1:
                lv += 1
        s = str(lv)
        t = s.rstrip("0")
        return t, dec + len(s)
    dec_exp = _estimate_dec_exp(fract, bin_exp)
    B5 = max(0, -dec_exp)
    B2 = B5 + ntiny + bin_exp
    S5 = max(0, dec_exp)
    S2 = S5 + ntiny
    M5, M2 = B5, B2 - nsig
    fb = fract >> tail
    B2 -= nfract - 1
    c2 = min(B2, S2)
    B2, S2, M2 = B2 - c2, S2 - c2, M2 - c2
    if nfract == 1:
        M2 -= 1
    if M2 < 0:
        B2, S2, M2 = B2 - M2, S2 - M2, 0
    bbits = nfract + B2 + (_n5bits(B5) if B5 < 27 else B5 * 3)
    tsbits = S2 + 1 + (_n5bits(S5 + 1) if S5 + 1 < 27 else (S5 + 1) * 3)
    digits = []
    if bbits < 64 and tsbits < 64:
        wrap = _i32 if (bbits < 32 and tsbits < 32) else _i64
        b = (fb * 5 ** B5) << B2
        s = 5 ** S5 << S2
        m = 5 ** M5 << M2
        tens = s * 10
        q, b = b // s, 10 * (b % s)
        m = wrap(m * 10)
        low, high = b < m, wrap(b + m) > tens
        if q == 0 and not high:
            dec_exp -= 1
        else:
            digits.append(q)
        if dec_exp < -3 or dec_exp >= 8:
            low = high = False
        while not low and not high:
            q, b = b // s, 10 * (b % s)
            m = wrap(m * 10)
            if m > 0:
                low, high = b < m, wrap(b + m) > tens
            else:  # the JDK's overflow "hack"
                low = high = True
            digits.append(q)
        ldd = wrap((b << 1) - tens)
    else:
        S = 5 ** S5 << S2
        B = (fb * 5 ** B5) << B2
        M = 5 ** (M5 + 1) << (M2 + 1)
        TS = 5 ** (S5 + 1) << (S2 + 1)
        q, B = B // S, (B % S) * 10
        low, high = B < M, B + M >= TS
        if q == 0 and not high:
            dec_exp -= 1
        else:
            digits.append(q)
        if dec_exp < -3 or dec_exp >= 8:
            low = high = False
        while not low and not high:
            q, B = B // S, (B % S) * 10
            M *= 10
            low, high = B < M, B + M >= TS
            digits.append(q)
        ldd = ((B << 1) > TS) - ((B << 1) < TS) if (high and low) else 0
    dec = dec_exp + 1
    if high and (not low or ldd > 0 or (ldd == 0 and digits[-1] & 1)):
        i = len(digits) - 1  # roundup(): carry through trailing nines
        while digits[i] == 9 and i > 0:
            digits[i] = 0
            i -= 1
        if digits[i] == 9:  # all nines: "1" and a larger exponent, the zeros stay as digits
            digits[0] = 1
            dec += 1
        else:
            digits[i] += 1
    return "".join(chr(48 + v) for v in digits), dec


def jdk8_double_string(d: float) -> str:
    """java.lang.Double.toString(d) as JDK 7/8 print it."""
    u = _bits(d)
    neg = u >> 63
    fract = u & ((1 << 52) - 1)
    be = (u >> 52) & 0x7FF
    if be == 0x7FF:
        return "NaN" if fract else ("-Infinity" if neg else "Infinity")
    if be == 0:
        if fract == 0:
            return "-0.0" if neg else "0.0"
        lz = 64 - fract.bit_length()
        shift = lz - 11
        fract <<= shift
        be = 1 - shift
        nsig = 64 - lz
    else:
        fract |= 1 << 52
        nsig = 53
    digs, e = _dtoa(be - 1023, fract, nsig)
    out = "-" if neg else ""
    n = len(digs)
    if 0 < e < 8:
        k = min(n, e)
        out += digs[:k]
        if k < e:
            out += "0" * (e - k) + ".0"
        else:
            out += "." + (digs[k:] if k < n else "0")
    elif -3 < e <= 0:
        out += "0." + "0" * (-e) + digs
    else:
        out += digs[0] + "." + (digs[1:] if n > 1 else "0") + "E" + str(e - 1)
    return out


# ------------------------------------------------------------------------------------------
# Scala 2.10 hashing: the iteration order of `splits.toSet` (EvenSplitPartitioner.scala:161)
# ------------------------------------------------------------------------------------------
def _rotl(v: int, r: int) -> int:
    v &= _M32
    return ((v << r) | (v >> (32 - r))) & _M32


def _mix_last(h: int, k: int) -> int:
    k = (k * 0xCC9E2D51) & _M32
    k = _rotl(k, 15)
    k = (k * 0x1B873593) & _M32
    return (h ^ k) & _M32


def _mix(h: int, k: int) -> int:
    h = _rotl(_mix_last(h, k), 13)
    return (h * 5 + 0xE6546B64) & _M32


def _avalanche(h: int) -> int:
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & _M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & _M32
    h ^= h >> 16
    return h


def _java_d2i(d: float) -> int:  # Java (int) of a double: truncation, saturation, NaN -> 0
    if d != d:
        return 0
    if d >= 2147483647.0:
        return 2147483647
    if d <= -2147483648.0:
        return -2147483648
    return int(d)


def _java_d2l(d: float) -> int:  # Java (long) of a double
    if d != d:
        return 0
    if d >= 9.223372036854775807e18:
        return (1 << 63) - 1
    if d <= -9.223372036854775808e18:
        return -(1 << 63)
    return int(d)


def hash_from_double(d: float) -> int:
    """scala.runtime.BoxesRunTime.hashFromDouble (a boxed Double's ##), as an unsigned 32-bit
    value: the int value if it is exact, else the long's hashCode, else the float's, else the
    double's."""
    iv = _java_d2i(d)
    if float(iv) == d:
        return iv & _M32
    lv = _java_d2l(d)
    if float(lv) == d:
        u = lv & ((1 << 64) - 1)  # Long.hashCode: (int) (v ^ (v >>> 32))
        return (u ^ (u >> 32)) & _M32
    f = struct.unpack("<f", struct.pack("<f", d))[0] if abs(d) <= 3.4028234663852886e38 else (
        float("inf") if d > 0 else float("-inf"))
    if f == d:  # Float.hashCode = floatToIntBits (finite here: d == f)
        return struct.unpack("<I", struct.pack("<f", f))[0]
    u = _bits(d)
    if d != d:
        u = 0x7FF8000000000000  # doubleToLongBits: the canonical NaN
    return (u ^ (u >> 32)) & _M32


def rect_hash(x: float, y: float, x2: float, y2: float) -> int:
    """DBSCANRectangle(x, y, x2, y2).hashCode: the case class hash of Scala 2.10,
    MurmurHash3.productHash(this) with productSeed 0xcafebabe, no product-prefix mixing."""
    h = 0xCAFEBABE
    for v in (x, y, x2, y2):
        h = _mix(h, hash_from_double(v))
    return _avalanche(h ^ 4)


def improve(h: int) -> int:
    """immutable.HashSet.improve (Scala 2.10), on the 32-bit hash."""
    h = _i32(h)
    h = _i32(h + ~_i32(h << 9))
    h = _i32(h ^ ((h & _M32) >> 14))
    h = _i32(h + _i32(h << 4))
    return (h ^ ((h & _M32) >> 10)) & _M32


def trie_key(ih: int) -> int:
    """HashTrieSet iteration rank of an improved hash: the trie branches on 5-bit groups from
    the lowest bits up and iterates each node's children in ascending index order, so elements
    come in lexicographic order of (bits 0-4, bits 5-9, ..., bits 30-31)."""
    k = 0
    for level in range(0, 30, 5):
        k = (k << 5) | ((ih >> level) & 31)
    return (k << 2) | (ih >> 30)


def split_order_key(x: float, y: float, x2: float, y2: float) -> int:
    """Rank of the candidate DBSCANRectangle(x, y, x2, y2) in the iteration order of a
    HashTrieSet (a `splits.toSet` of more than 4 candidates): smaller comes first."""
    return trie_key(improve(rect_hash(x, y, x2, y2)))
