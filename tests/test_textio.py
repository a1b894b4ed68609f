"""Text I/O of the reference (csrc/csv.hip) -- host code, CPU tests.

Input: DBSCANSuite.scala:31-33 (textFile + split(',') + toDouble, x/y = fields 0/1).
Output: DBSCANSample.scala:35 ("x,y,cluster" with java.lang.Double.toString)."""
import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN
from dbscan_amd import DBSCANError
from dbscan_amd.textio import format_double, read_csv, write_csv


def test_read_labeled_data_csv():
    x, y = read_csv(f"{GOLDEN}/labeled_data.csv")
    rx, ry, _ = O.load_labeled_csv(f"{GOLDEN}/labeled_data.csv")
    assert x.size == 749
    np.testing.assert_array_equal(x, rx)
    np.testing.assert_array_equal(y, ry)


@pytest.mark.parametrize("v,s", [
    (1.0, "1.0"), (-2.5, "-2.5"), (0.001, "0.001"), (1e-4, "1.0E-4"), (1e7, "1.0E7"),
    (9999999.0, "9999999.0"), (123456.789, "123456.789"), (0.0, "0.0"), (-0.0, "-0.0"),
    (float("nan"), "NaN"), (float("inf"), "Infinity"), (float("-inf"), "-Infinity"),
    (0.30000001192092896, "0.30000001192092896"), (1.7976931348623157e308,
                                                    "1.7976931348623157E308"),
    (4.9e-324, "4.9E-324"), (100.0, "100.0"), (1.5e-3, "0.0015"), (2.0e22, "2.0E22")])
def test_java_double_to_string(v, s):
    """java.lang.Double.toString layout (JDK shortest digits)."""
    assert format_double(v) == s


def test_round_trip_and_reference_output_format(tmp_path):
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.normal(size=500) * 10.0 ** rng.integers(-6, 9, 500),
                        [0.0, -0.0, 1e-3, 1e7]])
    y = rng.normal(size=x.size)
    cl = rng.integers(0, 9, x.size).astype(np.int32)
    p = tmp_path / "out.csv"
    write_csv(p, x, y, cl)
    lines = p.read_text().splitlines()
    assert lines[0] == f"{format_double(x[0])},{format_double(y[0])},{cl[0]}"
    rx, ry = read_csv(p)  # the label column parses and is ignored
    np.testing.assert_array_equal(rx.view(np.int64), x.view(np.int64))  # bit-exact, -0.0 too
    np.testing.assert_array_equal(ry, y)


def test_java_parse_forms(tmp_path):
    p = tmp_path / "in.csv"
    p.write_text(" 1.5 ,-2d,7\r\n+3e2,0x1.8p1,\nNaN,Infinity\n-Infinity,.5f,1,\n\n", "ascii")
    with pytest.raises(DBSCANError):  # the empty 5th line is a record: "".toDouble throws
        read_csv(p)
    p.write_text(" 1.5 ,-2d,7\r\n+3e2,0x1.8p1,\nNaN,Infinity\n-Infinity,.5f,1,\n", "ascii")
    x, y = read_csv(p)
    assert x[0] == 1.5 and y[0] == -2.0 and x[1] == 300.0 and y[1] == 3.0
    assert np.isnan(x[2]) and y[2] == np.inf and x[3] == -np.inf and y[3] == 0.5


@pytest.mark.parametrize("text", ["1.0\n", "1.0,abc\n", "1,2\ninf,3\n", "1,2,x\n", "1,,2\n"])
def test_malformed_records_raise(tmp_path, text):
    p = tmp_path / "bad.csv"
    p.write_text(text, "ascii")
    with pytest.raises(DBSCANError):
        read_csv(p)


def test_large_file_parallel_parse(tmp_path):
    rng = np.random.default_rng(2)
    n = 300_000
    x, y = rng.normal(size=n) * 1e3, rng.normal(size=n)
    p = tmp_path / "big.csv"
    write_csv(p, x, y, np.zeros(n, np.int32))
    rx, ry = read_csv(p)
    np.testing.assert_array_equal(rx, x)
    np.testing.assert_array_equal(ry, y)


# ------------------------- JDK 7/8 digits and Scala 2.10 ranges ---------------------------
@pytest.mark.parametrize("v,s", [
    # the JDK 19 release note for JDK-4511638: "Double.toString(2e23) now returns 2.0E23,
    # whereas in earlier releases it returns 1.9999999999999998E23"
    (2e23, "1.9999999999999998E23"),
    # the same symmetric-stopping-test path (FloatingDecimal's long branch)
    (1e23, "9.999999999999999E22"), (8.41e21, "8.409999999999999E21"),
    # the integer fast path keeps the digits above the half-ulp's "insignificant" ones
    (2.82879384806159e17, "2.82879384806159008E17"), (2.0 ** 62, "4.6116860184273879E18"),
    (2.0 ** 63, "9.223372036854776E18"), (1e17, "1.0E17"), (123456789012345680.0,
                                                              "1.2345678901234568E17")])
def test_jdk8_double_to_string_digits(v, s):
    """Spark 2.1.0 / Scala 2.10 run on JDK 7/8 (pom.xml:30-37), whose Double.toString
    (sun.misc.FloatingDecimal) prints more than the shortest digits for some values."""
    assert format_double(v) == s


def test_jvm_printed_doubles_from_reference_comments():
    """Every number the reference's own JVM printed into its source comments (golden data,
    tests/golden/jvm_printed_doubles.txt) is printed back identically."""
    vals = [l.split()[0] for l in open(f"{GOLDEN}/jvm_printed_doubles.txt") if l[0] != "#"]
    assert len(vals) > 50
    for s in vals:
        assert format_double(float(s)) == s, s


def test_jdk8_digits_round_trip_and_only_lengthen():
    """On random bit patterns: the printed value parses back to the same double, and the JDK
    7/8 digits are never shorter than the shortest round-trip digits (they equal them for all
    but a fraction of a percent of doubles)."""
    rng = np.random.default_rng(5)
    bits = rng.integers(0, 2 ** 63, 40_000, dtype=np.int64).view(np.float64)
    longer = 0
    for v in bits:
        if not np.isfinite(v):
            continue
        s = format_double(float(v))
        assert float(s) == v
        sig = lambda t: len(t.lstrip("-").split("E")[0].split("e")[0].replace(".", "").strip("0"))  # noqa
        assert sig(s) >= sig(repr(float(v)))
        longer += sig(s) > sig(repr(float(v)))
    assert longer < 0.01 * bits.size


@pytest.mark.parametrize("start,end,step,n", [
    (0.0, 0.9, 0.3, 3),   # decimal 0.9 / 0.3 = 3 exactly; exact binary division gives 3.0000..4 -> 4
    (0.0, 0.3, 0.1, 3), (0.6, 2.4, 0.6, 3), (1.0, 1.0, 0.5, 0), (2.0, 1.0, 0.5, 0),
    (-2.4, 2.4, 0.6000000238418579, 8), (0.1, 0.7, 0.2, 3)])
def test_scala_double_range_count_known(start, end, step, n):
    from dbscan_amd.partition import scala_range_count

    assert scala_range_count(start, end, step) == n == O.scala_range_count(start, end, step)


def test_scala_double_range_count_vs_oracle():
    """The product's NumericRange.count (csrc/javanum.hip: bigint decimal division) against
    the oracle's (Python decimal module) on grid-like and random ranges, until and to."""
    from dbscan_amd.partition import scala_range_count

    rng = np.random.default_rng(11)
    for _ in range(3000):
        mrs = float(2 * rng.choice([0.3, float(np.float32(0.3)), 2.55, 0.001, 1.7, 1e-5]))
        a, b = sorted(rng.integers(-5000, 5000, 2).tolist())
        start, end = a * mrs + mrs, b * mrs + rng.choice([0.0, mrs * 1e-9, -mrs * 1e-12])
        for inc in (False, True):
            if start == end or (start < end) != (mrs > 0):
                continue
            assert scala_range_count(start, end, mrs, inc) == O.scala_range_count(start, end, mrs,
                                                                                  inc)
    for _ in range(2000):
        start, end = rng.normal(size=2) * 10.0 ** rng.integers(-3, 4, 2)
        step = abs(rng.normal()) * 10.0 ** rng.integers(-3, 1)
        if end > start and (end - start) / step < 1e6:
            assert scala_range_count(start, end, step) == O.scala_range_count(start, end, step)


def test_double_to_string_two_restatements_agree():
    """java.lang.Double.toString as JDK 7/8 print it, restated twice: the product's
    csrc/javanum.hip (C++ bigints) and the oracle's oracle/jvm.py (Python ints), over random bit
    patterns, decimals of few digits, integers past 2^53 and tiny / huge magnitudes -- the digits
    BigDecimal(Double.toString(_)) sees in the partitioner's NumericRange count."""
    import random
    import struct

    import jvm

    from dbscan_amd.textio import format_double

    rng = random.Random(7)
    gens = [lambda: struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))[0],
            lambda: round(rng.uniform(-100, 100), rng.randint(0, 6)),
            lambda: rng.randint(-2 ** 62, 2 ** 62) * 1.0,
            lambda: rng.uniform(0, 1) * 10.0 ** rng.randint(-30, 30),
            lambda: 0.1 * rng.randint(-10000, 10000) + 2.0 * 0.30000001192092896]
    for g in gens:
        for _ in range(4000):
            v = g()
            assert format_double(v) == jvm.jdk8_double_string(v), repr(v)
