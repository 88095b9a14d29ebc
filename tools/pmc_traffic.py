"""Per-kernel HBM traffic from rocprofv3 --pmc counter_collection CSVs (FETCH_SIZE and
WRITE_SIZE passes), with the gfx950 FETCH_SIZE x2 correction (MI355X_MICROARCH.md §HBM).
usage: python tools/pmc_traffic.py fetch.csv write.csv [name-substring]"""
import collections
import csv
import sys


def load(path, counter):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        per[(r["Kernel_Name"][:90], r["Grid_Size"])].append(float(r["Counter_Value"]))
    return per


def main():
    f = load(sys.argv[1], "FETCH_SIZE")
    w = load(sys.argv[2], "WRITE_SIZE")
    sub = sys.argv[3] if len(sys.argv) > 3 else ""
    for k in f:
        if sub not in k[0]:
            continue
        fk = sum(f[k]) / len(f[k]) * 2.0  # KB; x2: gfx950 tallies 128-B requests at 64 B
        wk = sum(w.get(k, [0.0])) / max(1, len(w.get(k, [0.0])))
        print(f"{len(f[k]):4d} fetch {fk / 1024:9.2f} MB  write {wk / 1024:9.2f} MB  grid {k[1]:>8}  {k[0]}")


if __name__ == "__main__":
    main()
