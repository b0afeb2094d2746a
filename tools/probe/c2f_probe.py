"""Diagnostic: coarse-to-fine vs single-level LM on the rendered plane scene (prints costs and pose errors)."""
import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "oracle"), os.path.join(os.getcwd(), "tests")]
import numpy as np
import oracle as O
from helpers import engine_module, synth
E = engine_module()
for sigma in (0.002, 0.004, 0.008):
    pb = synth.make_problem(n_frames=10, n_points=1000, width=376, height=240, seed=41, border=16,
                            pose_sigma=sigma, rho_sigma=0.02)
    pb.poses[:2] = pb.poses_gt[:2]
    out, valid = O.evaluate(pb, poses=pb.poses_gt, rho=pb.rho_gt, want_jac=False)
    cgt = sum(O.huber_block(out[b, :pb.R], 9.0)[0] for b in range(pb.n_blocks) if valid[b])
    res = {}
    for mode in ("single", "pyramid"):
        with E.Engine(pb.kind, pb.model, huber_width=9.0) as eng:
            eng.set_problem(pb)
            eng.set_fixed_frames(np.array([0, 1], np.int32))
            eng.set_state(pb.poses, pb.rho)
            if mode == "pyramid":
                eng.build_pyramid(3)
                s = eng.solve_pyramid(max_iterations=15)
            else:
                s = eng.solve(max_iterations=45)
            poses, _ = eng.get_state()
        res[mode] = (s["initial_cost"], s["final_cost"], np.abs(poses[2:, 4:] - pb.poses_gt[2:, 4:]).max(1).mean(), s["iterations"])
    print(f"sigma {sigma}: gt cost {cgt:.1f}  err0 {np.abs(pb.poses[2:, 4:] - pb.poses_gt[2:, 4:]).max(1).mean():.5f}  {res}", flush=True)
