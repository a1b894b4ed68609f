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
