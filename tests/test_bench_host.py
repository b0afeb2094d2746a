"""Host logic of bench.py that runs without a GPU: the live roofline.traffic measurement's counter parsing and the
algorithmic bytes per block."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_counter_bytes_per_launch_sums_dimensions_and_averages_dispatches():
    b = _bench()
    k = b.HEADLINE_KERNEL
    rows = [
        # dispatch 1: two instance rows (summed), dispatch 2: one row; another kernel and another counter are ignored
        {"Dispatch_Id": "1", "Kernel_Name": f"void (anonymous namespace)::{k}(pba::detail::KernelArgs)",
         "Counter_Name": "FETCH_SIZE", "Counter_Value": "100.0"},
        {"Dispatch_Id": "1", "Kernel_Name": f"void (anonymous namespace)::{k}(pba::detail::KernelArgs)",
         "Counter_Name": "FETCH_SIZE", "Counter_Value": "50.0"},
        {"Dispatch_Id": "2", "Kernel_Name": f"void (anonymous namespace)::{k}(pba::detail::KernelArgs)",
         "Counter_Name": "FETCH_SIZE", "Counter_Value": "250.0"},
        {"Dispatch_Id": "3", "Kernel_Name": "void linearize_kernel<0, 0, 8>(...)", "Counter_Name": "FETCH_SIZE",
         "Counter_Value": "9999.0"},
        {"Dispatch_Id": "2", "Kernel_Name": f"{k}", "Counter_Name": "WRITE_SIZE", "Counter_Value": "7.0"},
    ]
    assert b.counter_bytes_per_launch(rows, "FETCH_SIZE", k) == (150.0 + 250.0) / 2 * 1024.0
    assert b.counter_bytes_per_launch(rows, "WRITE_SIZE", k) == 7.0 * 1024.0
    assert b.counter_bytes_per_launch(rows, "GRBM_COUNT", k) is None


def test_algorithmic_bytes_per_block_at_c4():
    b = _bench()
    # 517.3 B at P = 8, K = 4 on the C4 problem
    v = b.algorithmic_bytes_per_block(8, 4, 1004, 100000, 400000)
    assert abs(v - 517.28) < 0.01
