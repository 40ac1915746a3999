import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE / "golden"))
sys.path.insert(0, str(HERE.parent))

# GPU test modules whose kernels (or host paths feeding them) have not yet run on an
# MI355X run after the rest of the suite, so that under `pytest -x` a failure there
# cannot hide the results of the validated kernels.  test_bam2cns_cli.py: its BAM input
# now goes through the native decoder (pr_bam_decode_alns; CPU-checked field for field).
RUN_LAST = ("test_bam2cns_cli.py", "test_fantasticus_cns.py", "test_mask_gpu.py", "test_seed_gpu.py", "test_correct_loop.py",
            "test_sw_edge_gpu.py", "test_perl_xs.py", "test_perl_xs_mem.py", "test_file_chain_gpu.py")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libprgpu.so on the device)")


def pytest_collection_modifyitems(session, config, items):
    def rank(it):
        name = Path(str(it.fspath)).name
        return RUN_LAST.index(name) + 1 if name in RUN_LAST else 0
    items.sort(key=rank)
