"""scripts/rocpd_stats.py --exclusive: overlapped kernel time split evenly among the kernels that
share it, so family shares add up to the GPU-busy time (the union of the intervals)."""
import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exclusive_shares(tmp_path):
    db = tmp_path / "t.db"
    c = sqlite3.connect(db)
    c.execute("create table kernels(name text, start int, end int)")
    c.executemany("insert into kernels values(?,?,?)", [
        ("void mxs::paged_decode_mfma_kernel<64, 4, 2>(int)", 0, 100),   # alone 0-50, shared 50-100
        ("void mxs::paged_prefill_v3_kernel<64, 4, 2, 0>(int)", 50, 150),  # shared 50-100, alone 100-150
        ("Cijk_Alik_Bljk_MT256x256", 200, 300),                          # alone
        ("Custom_Cijk_Alik_Bljk_SK3", 300, 350)])                        # alone, same family
    c.commit()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rocpd_stats.py"), str(db), "--exclusive"],
                         capture_output=True, text=True, check=True).stdout
    rows = {ln.split()[-1]: (float(ln.split()[0][:-1]), float(ln.split()[1][:-1]))
            for ln in out.splitlines() if not ln.startswith("#")}
    # busy = 300 ns: decode 75, prefill 75, hipblaslt 150; raw = 350 ns
    assert rows["hipblaslt"][0] == 50.0 and abs(rows["mxs::paged_decode_mfma_kernel"][0] - 25.0) < 1e-6
    assert abs(rows["mxs::paged_prefill_v3_kernel"][0] - 25.0) < 1e-6
    assert abs(sum(v[0] for v in rows.values()) - 100.0) < 0.05
    assert "overlap 16.7 %" in out
