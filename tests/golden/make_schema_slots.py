#!/usr/bin/env python3
"""Generate tests/golden/schema_slots.json from the reference's generated
FlatBuffers code (/root/reference/src/schema_generated.rs, flatc output for
src/schema.fbs).  Run in the build container, where the reference exists:

    python tests/golden/make_schema_slots.py

The fixture records, as data, what the .rten format defines -- enum values
(OperatorType, OperatorAttrs union ids, NodeKind, ConstantData, Scalar,
AutoPad, DataType, ConstantDataType) and, per table, every field's vtable slot
((VT_x - 4) / 2), scalar type and default -- so tests/test_schema_pin.py can
check the writer (rten_hip/rten_file.py) and the loader (csrc/model.cpp)
against the format instead of against each other.
"""
import json
import os
import re
import sys

SRC = "/root/reference/src/schema_generated.rs"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "schema_slots.json")


def parse(text):
    enums = {}
    for m in re.finditer(r"^impl (\w+) \{\n((?:    pub const \w+: Self = Self\(-?\d+\);\n)+)", text, re.M):
        enums[m.group(1)] = {k: int(v) for k, v in re.findall(r"pub const (\w+): Self = Self\((-?\d+)\);",
                                                             m.group(2))}
    tables = {}
    for m in re.finditer(r"^impl<'a> (\w+)<'a> \{\n(.*?)^}\n", text, re.M | re.S):
        name, body = m.group(1), m.group(2)
        vts = dict(re.findall(r"pub const VT_(\w+): flatbuffers::VOffsetT = (\d+);", body))
        if not vts:
            continue
        fields = {}
        for vt, off in vts.items():
            f = {"slot": (int(off) - 4) // 2}
            g = re.search(r"\.get::<([^>(]+?(?:<[^;]*?>)?)>\(\s*%s::VT_%s,\s*(None|Some\(([^)]*)\))" % (name, vt),
                          body, re.S)
            if g:
                ty, dflt = g.group(1).strip(), g.group(3)
                f["type"] = "ref" if "ForwardsUOffset" in ty else ty
                if dflt is not None:
                    f["default"] = dflt.strip()
            fields[vt.lower()] = f
        tables[name] = fields
    return enums, tables


def main():
    if not os.path.exists(SRC):
        sys.exit(f"{SRC} not found (run this in the build container)")
    enums, tables = parse(open(SRC).read())
    json.dump({"source": "src/schema_generated.rs (flatc output of src/schema.fbs)",
               "enums": enums, "tables": tables}, open(OUT, "w"), indent=1, sort_keys=True)
    print(f"wrote {OUT}: {len(enums)} enums, {len(tables)} tables")


if __name__ == "__main__":
    main()
