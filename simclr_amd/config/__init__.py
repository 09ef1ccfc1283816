from .compose import (Config, Composer, ConfigCompositionError, compose, get_original_cwd,
                      hydra_main, load_yaml_text, parse_value, run_job, task_config, to_yaml,
                      to_absolute_path)
from .validate import check_pretrain_conf, check_eval_conf, check_save_features_conf, \
    check_supervised_conf

CONF_DIR = __import__("pathlib").Path(__file__).resolve().parents[2] / "conf"

__all__ = ["Config", "Composer", "ConfigCompositionError", "compose", "get_original_cwd",
           "hydra_main", "load_yaml_text", "parse_value", "run_job", "task_config", "to_yaml",
           "to_absolute_path", "check_pretrain_conf", "check_eval_conf",
           "check_save_features_conf", "check_supervised_conf", "CONF_DIR"]
