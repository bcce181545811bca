"""The reference's entry-point scripts run end to end on CPU (tiny sizes): train_ioi.py -> eval_ioi.py."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_train_then_eval_ioi(tmp_path):
    import eval_ioi
    import train_ioi
    root = str(tmp_path / "models" / "ioi")
    train_ioi.main(["--num-samples", "96", "--epochs", "1", "--batch-size", "32", "--save-root", root,
                    "--max-steps", "2", "--no-early-stop"])
    d = os.path.join(root, "IOI_ModelPair", "100_100_40")
    assert os.path.exists(os.path.join(d, "ll_model.pth"))
    df = eval_ioi.main(["-w", "100_100_40", "--root", root, "--num-samples", "64", "-b", "32",
                        "--resample-batch-size", "32", "-m", "true"])
    assert set(df["status"]) == {"in_circuit", "not_in_circuit"}
    assert len(df) == 8 + 7
    assert os.path.exists(os.path.join(d, "results", "results.csv"))
    assert os.path.exists(os.path.join(d, "results", "metric_collection.log"))


def test_pvr_scripts(tmp_path):
    import eval_causality
    import eval_information
    import train as train_pvr
    hp = ["mod.layer3.mod.1.mod.conv2.hook_point"]
    pair = train_pvr.main(["--train-size", "32", "--test-size", "16", "--epochs", "1", "--batch-size", "16",
                           "--save", str(tmp_path / "w.pt")])
    assert (tmp_path / "w.pt").exists()
    stats = eval_causality.main(["--weights", str(tmp_path / "w.pt"), "--test-size", "16", "--batch-size", "8",
                                 "--hook-points", *hp, "--out-dir", str(tmp_path / "plots")])
    assert len(stats[hp[0]]) == 12 and all(0 <= v <= 1 for v in stats[hp[0]].values())
    correct, leaky, leaky_all = eval_information.main(
        ["--train-size", "32", "--test-size", "16", "--epochs", "1", "--batch-size", "16", "--probe-batch-size", "16",
         "--hook-points", *hp, "--out-dir", str(tmp_path / "plots")])
    assert correct.shape == (1, 4) and leaky.shape == (1, 4) and leaky_all.shape == (1, 12)
    assert (tmp_path / "plots" / "bin" / "leaky_accs_all.npy").exists()
