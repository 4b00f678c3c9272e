"""tools/pmc_summary.py: the roofline's `traffic` comes from it (bench.py reads
profiles/pmc_summary.json), so its byte arithmetic is checked on synthetic
rocprofv3 counter CSVs: FETCH_SIZE doubled, WRITE_SIZE in KB, and -- with the
request-size pass -- read bytes as 32 / 64 / 128 B per request, which then
replace the doubled FETCH_SIZE (exact for any request mix)."""
import csv
import importlib.util
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
spec = importlib.util.spec_from_file_location("pmc_summary", ROOT / "tools" / "pmc_summary.py")
pmc_summary = importlib.util.module_from_spec(spec)
spec.loader.exec_module(pmc_summary)

K = "void dqdk::rx_decode_fused_kernel<2, false, false>(dqdk::RxArgs)"


def write_pass(d: Path, name: str, rows):
    p = d / name / "run_counter_collection.csv"
    p.parent.mkdir(parents=True)
    with open(p, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for disp, c, v in rows:
            w.writerow({"Dispatch_Id": disp, "Kernel_Name": K, "Counter_Name": c, "Counter_Value": v})


def test_fetch_write_only(tmp_path):
    write_pass(tmp_path, "p1", [(1, "FETCH_SIZE", 1000.0), (2, "FETCH_SIZE", 1200.0)])
    write_pass(tmp_path, "p2", [(3, "WRITE_SIZE", 50.0), (4, "WRITE_SIZE", 50.0)])
    m = pmc_summary.summarise(tmp_path)["rx_decode_fused_kernel"]
    assert m["dispatches"] == 2
    assert m["hbm_read_bytes_corrected"] == m["hbm_read_bytes_fetch_x2"] == 1100.0 * 1024 * 2
    assert m["hbm_bytes_per_launch"] == 1100.0 * 2048 + 50.0 * 1024
    assert "hbm_read_bytes_by_size" not in m


def test_request_sizes_replace_the_doubling(tmp_path):
    write_pass(tmp_path, "p1", [(1, "FETCH_SIZE", 2000.0)])
    write_pass(tmp_path, "p2", [(2, "WRITE_SIZE", 10.0)])
    write_pass(tmp_path, "p4", [(3, "TCC_EA0_RDREQ_sum", 1000.0), (3, "TCC_EA0_RDREQ_32B_sum", 100.0),
                                (3, "TCC_EA0_RDREQ_64B_sum", 300.0), (3, "TCC_EA0_RDREQ_128B_sum", 600.0)])
    m = pmc_summary.summarise(tmp_path)["rx_decode_fused_kernel"]
    exact = 32 * 100 + 64 * 300 + 128 * 600
    assert m["hbm_read_bytes_by_size"] == exact
    assert m["rdreq_unsized"] == 0
    assert m["hbm_read_bytes_corrected"] == exact
    assert m["hbm_read_bytes_fetch_x2"] == 2000.0 * 2048
    assert m["hbm_bytes_per_launch"] == exact + 10.0 * 1024
