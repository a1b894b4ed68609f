"""Register, LDS and instruction counts of kernels in a device assembly listing
(`make -C dbscan-on-spark_amd/csrc asm OUT=/tmp/x` writes /tmp/x/asm/fit.s):
    python tools/asm_stats.py /tmp/x/asm/fit.s count_tile32 [--dump]
--dump prints the matching kernels' instruction bodies (labels kept, directives dropped)."""
import re
import sys


def kernels(text, pat):
    for m in re.finditer(r"^(_Z\S+):\s*;\s*@", text, re.M):
        name = m.group(1)
        if pat not in name:
            continue
        end = text.index(".Lfunc_end", m.end())
        body = text[m.end():end]
        tail = text[end:end + 6000]

        def num(key):
            mm = re.search(re.escape(name) + r"\." + key + r",\s*(\d+)", text)
            return int(mm.group(1)) if mm else None

        lds = re.search(r"\.amdhsa_group_segment_fixed_size\s+(\d+)", text[text.index(".amdhsa_kernel " + name):])
        scratch = re.search(r"\.amdhsa_private_segment_fixed_size\s+(\d+)", text[text.index(".amdhsa_kernel " + name):])
        yield name, body, {"vgpr": num("num_vgpr"), "sgpr": num("numbered_sgpr"),
                           "lds": int(lds.group(1)) if lds else None,
                           "scratch": int(scratch.group(1)) if scratch else None}, tail


def main():
    path, pat = sys.argv[1], sys.argv[2]
    text = open(path).read()
    for name, body, meta, _ in kernels(text, pat):
        ins = [l.strip() for l in body.split("\n")]
        ins = [l for l in ins if l and not l.startswith((".", ";")) and not l.endswith(":")]
        kinds = {}
        for l in ins:
            op = l.split()[0]
            k = op.split("_")[0]
            kinds[k] = kinds.get(k, 0) + 1
        short = re.sub(r"^_ZN6dbscan12_GLOBAL__N_1\d+", "", name)[:70]
        print(f"{short}: {len(ins)} instrs {meta} by prefix {dict(sorted(kinds.items(), key=lambda t: -t[1]))}")
        if "--dump" in sys.argv:
            for l in body.split("\n"):
                s = l.strip()
                if s and not s.startswith("."):
                    print(l)


if __name__ == "__main__":
    main()
