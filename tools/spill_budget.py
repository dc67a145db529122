"""Register-spill report of the shipped library's kernels, from the code-object notes (amdhsa.kernels:
.private_segment_fixed_size, .sgpr_spill_count, .vgpr_spill_count).

  python tools/spill_budget.py            # print every kernel that spills
  python tools/spill_budget.py --write    # commit the current figures as tests/spill_budget.json

tests/test_abi.py::test_spill_budget fails when any kernel exceeds its committed figures (a kernel not in
the budget has budget 0)."""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
BUDGET = os.path.join(ROOT, "tests", "spill_budget.json")
KEYS = ("private_segment_fixed_size", "sgpr_spill_count", "vgpr_spill_count")


def kernel_spills(so_path):
    """{mangled kernel name: {key: int}} for every gfx950 kernel bundled in so_path's .hip_fatbin."""
    d = tempfile.mkdtemp()
    fat = os.path.join(d, "fat.bin")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", so_path, fat], check=True)
    data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)] + [len(data)]
    out = {}
    for i in range(len(starts) - 1):
        part = os.path.join(d, f"b{i}.bin")
        with open(part, "wb") as f:
            f.write(data[starts[i]:starts[i + 1]])
        dev = os.path.join(d, f"b{i}.o")
        r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}", f"--output={dev}",
                            "--unbundle"], capture_output=True)
        if r.returncode or not os.path.exists(dev) or os.path.getsize(dev) == 0:
            continue
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", dev], capture_output=True,
                               text=True, check=True).stdout
        # one YAML mapping per kernel: its keys come before or after .name, so collect per "- " item
        for item in re.split(r"\n\s*- \.", "\n" + notes.split("amdhsa.kernels:", 1)[-1]):
            m = re.search(r"(?:^|\n)\s*\.?name:\s*(\S+)", item)
            if not m or m.group(1).endswith(".kd"):
                continue
            rec = {}
            for k in KEYS:
                mk = re.search(r"(?:^|\n)\s*\.?%s:\s*(\d+)" % k, item)
                rec[k] = int(mk.group(1)) if mk else 0
            out[m.group(1)] = rec
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.split("\n") if r.returncode == 0 else list(names)


def main():
    so = os.path.join(ROOT, "superresolution_for_pdes_amd", "lib", "libsrpde_hip.so")
    ks = kernel_spills(so)
    spilling = {k: v for k, v in sorted(ks.items()) if any(v.values())}
    if "--write" in sys.argv:
        with open(BUDGET, "w") as f:
            json.dump({"_doc": "per-kernel spill budget (tools/spill_budget.py); kernels not listed: 0",
                       "kernels": spilling}, f, indent=1, sort_keys=True)
        print(f"wrote {BUDGET}: {len(spilling)} of {len(ks)} kernels spill")
    for name, dn in zip(spilling, demangle(list(spilling))):
        v = spilling[name]
        print(f"{v['private_segment_fixed_size']:5d} B scratch {v['sgpr_spill_count']:4d} SGPR {v['vgpr_spill_count']:4d} VGPR  {dn}")


if __name__ == "__main__":
    main()
