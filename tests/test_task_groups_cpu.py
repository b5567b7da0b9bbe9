"""Task-group planning for second-order meta-steps (maml.plan_task_group): groups are the
largest that keep every inner step's primal resident, balanced; pure host logic."""
from weatherforecast_stgcn_maml_amd.config import CONFIG1, CONFIG2, CONFIG5, MamlConfig
from weatherforecast_stgcn_maml_amd.maml import KEEP_MARGIN, plan_task_group, task_bytes

GIB = 1 << 30
HBM = 268 * GIB  # an MI355X's 288 GB


def test_task_bytes_config2():
    cfg = MamlConfig(inner_steps=5, batch=32, order=2)
    # workspace 9.4 GB + feature cache 1.7 GB + kept primal (dG+dh, then 4 x Hs/Cs/Gs/dG/dh)
    assert abs(task_bytes(CONFIG2, cfg, 5) / 1e9 - 45.1) < 0.2
    assert task_bytes(CONFIG2, cfg, 0) < task_bytes(CONFIG2, cfg, 1) < task_bytes(CONFIG2, cfg, 5)


def test_groups_balanced_and_fit():
    cfg = MamlConfig(inner_steps=5, batch=32, order=2)
    per = task_bytes(CONFIG2, cfg, 5)
    for n, want in ((15, 5), (8, 4), (7, 4), (4, 4), (2, 2), (1, 1)):
        g = plan_task_group(CONFIG2, cfg, n, HBM)
        assert g == want, (n, g)
        assert g * per <= HBM - KEEP_MARGIN
        groups = -(-n // g)
        assert g * groups - n < groups  # balanced: no group is more than one task short


def test_first_order_and_small_configs_run_in_one_group():
    assert plan_task_group(CONFIG2, MamlConfig(order=1), 15, HBM) == 15
    assert plan_task_group(CONFIG1, MamlConfig(inner_steps=2, batch=2, order=2), 15, HBM) == 15


def test_config5_one_task_per_group():
    cfg = MamlConfig(inner_steps=10, batch=32, order=2)
    assert plan_task_group(CONFIG5, cfg, 8, HBM) == 1
