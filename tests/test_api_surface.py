"""every public symbol of the reference API resolves (through the ``iit`` alias package)."""
import importlib

import pytest

import iit  # noqa: F401  (installs the alias finder)

SURFACE = {
    "iit.model_pairs": ["BaseModelPair", "IITModelPair", "IITBehaviorModelPair", "StrictIITModelPair",
                        "FreezedModelPair", "StopGradModelPair", "IOI_ModelPair", "IITProbeSequentialPair",
                        "HLNode", "LLNode"],
    "iit.model_pairs.stop_grad_pair": ["StopGradHookedModel"],
    "iit.utils": ["IITDataset", "Ix", "HookedModuleWrapper", "DEVICE", "WANDB_ENTITY"],
    "iit.utils.index": ["TorchIndex", "Index", "Ix"],
    "iit.utils.correspondence": ["Correspondence"],
    "iit.utils.iit_dataset": ["IITDataset", "train_test_split"],
    "iit.utils.eval_datasets": ["IITUniqueDataset"],
    "iit.utils.metric": ["MetricType", "MetricStore", "PerTokenMetricStore", "MetricStoreCollection"],
    "iit.utils.node_picker": ["get_all_nodes", "get_nodes_in_circuit", "nodes_intersect", "get_nodes_not_in_circuit",
                              "get_post_nodes_not_in_circuit", "get_activation_idx", "get_params_in_circuit",
                              "get_all_params", "get_params_not_in_circuit", "LLParamNode"],
    "iit.utils.eval_ablations": ["Categorical_Metric", "do_intervention", "resample_ablate_node",
                                 "check_causal_effect", "get_mean_cache", "make_ablation_hook", "ablate_node",
                                 "get_causal_effects_for_all_nodes", "check_causal_effect_on_ablation",
                                 "make_dataframe_of_results", "make_combined_dataframe_of_results", "save_result"],
    "iit.utils.eval_metrics": ["kl_div", "accuracy_affected"],
    "iit.utils.probes": ["construct_probe", "construct_probes", "train_probes_on_model_pair", "evaluate_probe"],
    "iit.utils.plotter": ["plot_probe_stats", "plot_ablation_stats", "get_hookpoint_labels",
                          "get_leaky_hlnode_labels"],
    "iit.utils.wrapper": ["get_hook_points", "HookedModuleWrapper"],
    "iit.utils.logger": ["LoggingDict"],
    "iit.tasks.hl_model": ["HLModel"],
    "iit.tasks.task_loader": ["get_dataset", "get_alignment"],
    "iit.tasks.ioi": ["make_ioi_dataset_and_hl", "NAMES", "IOI_HL", "IOIDataset", "IOIDatasetWrapper", "n_layers",
                      "n_heads", "d_model", "d_head", "ioi_cfg", "all_attns", "all_mlps", "corr_dict", "suffixes",
                      "corr"],
    "iit.tasks.ioi.ioi_hl": ["DuplicateHead", "PreviousHead", "InductionHead", "SInhibitionHead", "NameMoverHead"],
    "iit.tasks.mnist_pvr": ["ImagePVRDataset", "MNIST_PVR_HL", "MNIST_PVR_Leaky_HL", "get_corr", "get_alignment",
                            "MNIST_CLASS_MAP"],
    "iit.tasks.mnist_pvr.utils": ["mnist_train", "mnist_test", "MNIST_CLASS_MAP"],
    "iit.tasks.docstring": ["Docstring_HL", "InductionHead", "ArgMoverHead"],
}

BASE_METHODS = ["loss_fn", "make_train_metrics", "make_test_metrics", "run_train_step", "run_eval_step",
                "do_intervention", "get_label_idxs", "make_hl_model", "set_corr", "sample_hl_name",
                "make_hl_ablation_hook", "hl_ablation_hook", "make_ll_ablation_hook", "get_IIT_loss_over_batch",
                "clip_grad_fn", "step_scheduler", "train", "make_loaders", "_run_train_epoch", "_run_eval_epoch",
                "_check_early_stop_condition", "_print_and_log_metrics"]


@pytest.mark.parametrize("module", sorted(SURFACE))
def test_symbols(module):
    if module == "iit.tasks.mnist_pvr.utils":
        mod = importlib.import_module(module)
        for name in SURFACE[module]:
            if name.startswith("mnist_"):
                continue  # built on first access (renders 60k digits); covered by test_mnist_pvr
            assert hasattr(mod, name), name
        return
    mod = importlib.import_module(module)
    for name in SURFACE[module]:
        assert hasattr(mod, name), f"{module}.{name}"


def test_base_model_pair_methods_and_subclass_extras():
    mp = importlib.import_module("iit.model_pairs")
    for m in BASE_METHODS:
        assert hasattr(mp.BaseModelPair, m), m
    assert hasattr(mp.IITBehaviorModelPair, "get_behaviour_loss_over_batch")
    assert hasattr(mp.IITBehaviorModelPair, "step_on_loss")
    assert hasattr(mp.StrictIITModelPair, "sample_ll_node")
    assert hasattr(mp.FreezedModelPair, "zero_grad_for_not_in_circuit")
    assert hasattr(mp.IOI_ModelPair, "_check_early_stop_fn")


def test_alias_objects_are_shared():
    from iit.utils.index import Ix as A
    from iit_amd.core.index import Ix as B
    assert A is B
