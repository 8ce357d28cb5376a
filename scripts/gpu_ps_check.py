"""Native parameter-server job on one MI355X: NUM_PS PS roles (default 1; 2 = the reference's
2 PS + workers shape, imagenet-resnet50-ps.py:75-84, with every variable range split over two
shards) + 2 workers as processes sharing the GPU through HIP IPC (on an 8-GPU node each role gets
its own GPU and the same mailboxes run over xGMI).  Every PS must apply every pushed step: a
multi-shard push / pull that lost or re-ordered a request shows up as a count mismatch.  Run
directly (the parent never touches the GPU before spawning the roles):

    NUM_PS=2 python scripts/gpu_ps_check.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    os.environ.setdefault("PDDL_PS", "impl=native,job_timeout=150")
    import pddl  # noqa: F401
    from pddl.config import make_config
    from pddl.parallel.parameter_server import run_ps_job
    steps = int(os.environ.get("STEPS", "12"))
    cfg = make_config("ps", device="cuda", data="synthetic", image_size=224, crop=224, flip=True, epochs=1,
                      verbose=0, save=False, train_images=4096, val_images=64, seed=1, steps_per_epoch=steps,
                      batch_size=int(os.environ.get("BATCH", "32")), validation_steps=1)
    t0 = time.time()
    nps = int(os.environ.get("NUM_PS", "1"))
    res = run_ps_job(cfg, num_ps=nps, num_workers=2, return_results=True)
    dt = time.time() - t0
    ps = [r for r in res if r[0] == "ps"]
    wk = [r for r in res if r[0] == "worker"]
    print("results:", res, flush=True)
    assert len(ps) == nps and len(wk) == 2, res
    assert all(r[4] == "native" for r in ps), ps
    assert all(r[2] == steps for r in ps) and sum(r[2] for r in wk) == steps, res   # every shard, every push
    hist = [r for r in wk if r[3]][0][3]
    assert hist[0]["loss"] > 0 and "val_loss" in hist[0], hist
    print(f"native PS job ok: {steps} async steps (batch {cfg.batch_size}) on {nps} PS + 2 workers in {dt:.1f}s "
          f"(incl. process start-up); worker steps {[r[2] for r in wk]}, updates per PS {[r[2] for r in ps]}",
          flush=True)


if __name__ == "__main__":
    main()
