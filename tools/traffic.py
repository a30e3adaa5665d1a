"""HBM traffic per launch of the batch kernel from rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE in their own passes; both reported in KiB).
gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes
of a wide coalesced stream, so it is doubled; WRITE_SIZE is exact for 16-B
stores (the result records); the 4-B digest stores are uncalibrated.
    python tools/traffic.py <pmc dir> [out.json]"""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import main as summary  # noqa: E402


def traffic(root):
    s = summary(root)
    fetch = 2.0 * s.get("FETCH_SIZE", 0.0) * 1024.0
    write = s.get("WRITE_SIZE", 0.0) * 1024.0
    return {"fetch_bytes": fetch, "write_bytes": write, "bytes_per_launch": fetch + write,
            "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB->B, mean per dispatch"}


if __name__ == "__main__":
    t = traffic(sys.argv[1])
    if len(sys.argv) > 4:
        t["config"], t["instances"] = int(sys.argv[3]), int(sys.argv[4])
    print(json.dumps(t))
    if len(sys.argv) > 2:
        json.dump(t, open(sys.argv[2], "w"), indent=1)
