import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE / "golden"))
sys.path.insert(0, str(HERE.parent))

# GPU test modules run in this order after every other one, so that under `pytest -x` a
# failure in newer code cannot hide the results of the validated kernels: first what was
# green on a driver box before, then the Perl XS boundary (never yet driver-observed), then
# round-2 additions, then round-3 additions.
RUN_LAST = ("test_bam2cns_cli.py", "test_fantasticus_cns.py", "test_mask_gpu.py", "test_correct_loop.py",
            "test_perl_xs.py", "test_perl_xs_mem.py",
            "test_seed_gpu.py", "test_sw_edge_gpu.py", "test_aln_gpu.py", "test_configs4_gpu.py",
            "test_file_chain_gpu.py",
            "test_comm.py", "test_product_configs_gpu.py")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libprgpu.so on the device)")


def pytest_collection_modifyitems(session, config, items):
    def rank(it):
        name = Path(str(it.fspath)).name
        return RUN_LAST.index(name) + 1 if name in RUN_LAST else 0
    items.sort(key=rank)
