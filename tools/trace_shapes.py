"""Group a rocprofv3 kernel_trace.csv by (kernel, grid, LDS) and print the average duration
in the order each group first appears.  usage: python tools/trace_shapes.py trace.csv [min_calls]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    min_calls = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    groups, order = {}, []
    for r in rows:
        key = (r["Kernel_Name"][:70], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"],
               r["LDS_Block_Size"])
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if key not in groups:
            groups[key] = []
            order.append(key)
        groups[key].append(d)
    for k in order:
        v = groups[k]
        if len(v) >= min_calls:
            print(f"{len(v):5d} {sum(v) / len(v) / 1e3:8.2f}us  grid=({k[1]},{k[2]},{k[3]}) lds={k[4]:>6}  {k[0]}")


if __name__ == "__main__":
    main()
