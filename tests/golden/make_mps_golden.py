"""Generates tests/golden/mps/solomon_bp_c101_model.json from the reference's
own fixture ortools/routing/testdata/solomon_bp_c101.pb (an MPModelProto next
to solomon_bp_c101.mps in the same testdata target). The .pb is decoded with a
minimal protobuf wire-format reader; field numbers follow
ortools/linear_solver/linear_solver.proto (MPModelProto 1 maximize,
2 objective_offset, 3 variable, 4 constraint, 5 name; MPVariableProto
1 lower_bound, 2 upper_bound, 3 objective_coefficient, 4 is_integer, 5 name;
MPConstraintProto 2 lower_bound, 3 upper_bound, 4 name, 6 var_index (packed),
7 coefficient (packed)). Run where /root/reference exists; the JSON is what
the tests read."""
import json
import math
import struct
import sys

INF = float("inf")


def varint(b, i):
    r = s = 0
    while True:
        x = b[i]
        i += 1
        r |= (x & 0x7F) << s
        s += 7
        if x < 0x80:
            return r, i


def fields(b):
    i = 0
    while i < len(b):
        key, i = varint(b, i)
        f, t = key >> 3, key & 7
        if t == 0:
            v, i = varint(b, i)
        elif t == 1:
            v = struct.unpack_from("<d", b, i)[0]
            i += 8
        elif t == 2:
            n, i = varint(b, i)
            v = b[i:i + n]
            i += n
        elif t == 5:
            v = struct.unpack_from("<f", b, i)[0]
            i += 4
        else:
            raise ValueError(f"wire type {t}")
        yield f, t, v


def packed_varints(b):
    out, i = [], 0
    while i < len(b):
        v, i = varint(b, i)
        out.append(v - (1 << 64) if v >= (1 << 63) else v)
    return out


def packed_doubles(b):
    return list(struct.unpack(f"<{len(b) // 8}d", b))


def enc(x):
    return "inf" if x == INF else "-inf" if x == -INF else x


def main(src, dst):
    data = open(src, "rb").read()
    model = {"maximize": False, "objective_offset": 0.0, "name": "", "variables": [],
             "constraints": []}
    for f, t, v in fields(data):
        if f == 1:
            model["maximize"] = bool(v)
        elif f == 2:
            model["objective_offset"] = v
        elif f == 5:
            model["name"] = v.decode()
        elif f == 3:
            var = {"lb": -INF, "ub": INF, "obj": 0.0, "is_integer": False, "name": ""}
            for g, _, w in fields(v):
                if g == 1: var["lb"] = w
                elif g == 2: var["ub"] = w
                elif g == 3: var["obj"] = w
                elif g == 4: var["is_integer"] = bool(w)
                elif g == 5: var["name"] = w.decode()
            model["variables"].append(var)
        elif f == 4:
            con = {"lb": -INF, "ub": INF, "name": "", "var_index": [], "coefficient": []}
            for g, tt, w in fields(v):
                if g == 2: con["lb"] = w
                elif g == 3: con["ub"] = w
                elif g == 4: con["name"] = w.decode()
                elif g == 6: con["var_index"] += packed_varints(w) if tt == 2 else [w]
                elif g == 7: con["coefficient"] += packed_doubles(w) if tt == 2 else [w]
            model["constraints"].append(con)
    for v in model["variables"]:
        v["lb"], v["ub"] = enc(v["lb"]), enc(v["ub"])
    for c in model["constraints"]:
        c["lb"], c["ub"] = enc(c["lb"]), enc(c["ub"])
    json.dump(model, open(dst, "w"), separators=(",", ":"))
    print(f"{len(model['variables'])} variables, {len(model['constraints'])} constraints")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else
         "/root/reference/ortools/routing/testdata/solomon_bp_c101.pb",
         sys.argv[2] if len(sys.argv) > 2 else "tests/golden/mps/solomon_bp_c101_model.json")
