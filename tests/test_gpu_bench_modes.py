"""GPU: bench.py's other launch modes run and verify (the default pipelined mode runs in the round-end bench and in
tests/test_gpu_multirank.py).  --graph 1 replays one captured step of the pipeline-1 form; --pipeline 0 / 1, --no-plan
(the products write their own address streams) and --encode-only are the A/B and diagnostic forms the DESIGN.md
records quote.  Reduced in size: 4 objects of config2's shape.
"""
import pytest

from test_gpu_multirank import run_bench

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", [["--graph", "1"], ["--pipeline", "0"], ["--pipeline", "1"], ["--no-plan"],
                                  ["--encode-only"], ["--variant", "7"]], ids=lambda m: "".join(m).strip("-"))
def test_bench_mode(mode):
    line = run_bench(["--objects", "4", "--steps", "3", "--warmup", "1", "--breakdown-steps", "4", "--no-cpu-baseline",
                      "--no-ceiling"] + mode)
    assert line["n_gpus"] == 1 and line["value"] > 0 and line["ms_per_step"] > 0
    assert line["breakdown"]["verified"] is True
    assert line["roofline"]["achieved"] > 0
    if "--graph" in mode:
        assert "captured HIP graph" in line["config"]["pipeline"]
        assert line["config"]["pipeline"].startswith("elimination on a side stream")
