"""CLI and results layer (ofdm_based_systems.main vs main.py:19-393 of the reference).

CPU tests pin ``ResultsManager`` against ``tests/golden/cli.json`` (made by
``tests/golden/make_cli_golden.py`` from the reference's own ResultsManager): the CSV
text after every upsert, image file names and the docs/figures mirror, the channel
directory naming for every settings file, and ``main()``'s return code / message for a
missing configuration.  ``SimulationRunner`` is exercised with stand-in simulations
(the GPU path is covered by the ``gpu`` test at the end), and its multi-rank mode on
gloo with two ranks.
"""

import json
import os
import shutil
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp
from PIL import Image

from conftest import GOLDEN, ROOT

sys.path.insert(0, GOLDEN)  # make_cli_golden: the fixture's input tables

from ofdm_based_systems import main as M
from ofdm_based_systems.configuration.models import Settings, SimulationSettings

G = json.load(open(os.path.join(GOLDEN, "cli.json")))


def test_csv_upsert_matches_reference(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    rm = M.ResultsManager(channel_name="severe_multipath")
    for (name, snr, ber), want in zip(G["upserts"], G["csv_after_step"]):
        rm.update_ber_csv(name, snr, ber)
        assert rm.csv_path.read_text() == want


def test_image_names_and_mirror_match_reference(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    from make_cli_golden import BER_RESULTS, IMAGES

    rm = M.ResultsManager(channel_name="severe_multipath")
    img = Image.new("RGB", (8, 8))
    got = [os.path.relpath(rm.save_constellation_plot(image=img, **kw), tmp_path) for kw in IMAGES]
    assert got == G["images"]
    assert os.path.relpath(rm.plot_ber_vs_snr(BER_RESULTS), tmp_path) == G["ber_plot"]
    assert os.path.relpath(rm.plot_ber_vs_snr([]), tmp_path) == G["ber_plot_empty"]
    mirrored = sorted(os.path.join(r, f) for r, _, fs in os.walk("docs") for f in fs)
    assert mirrored == G["mirrored"]
    for p in G["images"] + [G["ber_plot"]]:
        assert (tmp_path / p).stat().st_size > 0


def test_no_docs_mirror(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    rm = M.ResultsManager(channel_name="x", doc_figures_dir=None)
    rm.save_constellation_plot(Image.new("RGB", (4, 4)), "CP", "OFDM", "ZF", 4, "QAM", "UNIFORM", 1.0)
    assert rm.doc_channel_dir is None and not os.path.exists("docs")


def test_channel_names_match_reference():
    for f, want in G["channel_names"].items():
        s = SimulationSettings.from_json(os.path.join(ROOT, "config", f))
        assert M.channel_name_of(s) == want, f


def test_main_missing_config(tmp_path, monkeypatch, capsys):
    monkeypatch.chdir(tmp_path)
    assert M.main() == G["main_missing_config_rc"]
    assert capsys.readouterr().out == G["main_missing_config_stdout"]


class _FakeSim:
    """Stand-in for a Simulation: the results dict keys main.py reads (simulation/models.py:413-444)."""

    def __init__(self, snr):
        self.snr_db = snr
        self.process_group = None

    def run(self):
        return {"snr_db": self.snr_db, "bit_error_rate": 10.0 ** (-self.snr_db / 10 - 1),
                "bit_errors": int(self.snr_db), "total_bits": 1000, "papr_db": 8.0 + self.snr_db / 100,
                "title": "CP-OFDM-MMSE", "prefix_acronym": "CP", "modulator_type": "OFDM",
                "equalizator_type": "MMSE", "constellation_order": 64, "constellation_scheme": "QAM",
                "power_allocation_acronym": "UNIFORM", "constellation_plot": Image.new("RGB", (4, 4))}


def _settings(snrs, rng_mode="reference"):
    return SimulationSettings(num_bands=64, signal_noise_ratios=snrs, channel_model_path="x.npy",
                              channel_type="CUSTOM", num_symbols=64, rng_mode=rng_mode)


def test_runner_end_to_end_with_stub_simulations(tmp_path, monkeypatch, capsys):
    monkeypatch.chdir(tmp_path)
    snrs = [0.0, 10.0, 20.0]
    monkeypatch.setattr(M.Simulation, "create_from_simulation_settings",
                        classmethod(lambda cls, s: [_FakeSim(x) for x in s.signal_noise_ratios]))
    rm = M.ResultsManager(channel_name="severe_multipath")
    runner = M.SimulationRunner(Settings(project_name="P", version="1"), _settings(snrs), rm)
    res = runner.run_all()
    runner.process_results(res)
    out = capsys.readouterr().out
    assert "Created 3 simulation(s) to run" in out and "Average PAPR: 8.10 dB" in out
    lines = rm.csv_path.read_text().splitlines()
    assert lines[0] == "simulation_name,snr_db,bit_error_rate" and len(lines) == 4
    assert lines[1].startswith("CP-OFDM-MMSE,0.0,")
    pngs = sorted(os.listdir(rm.images_dir))
    assert pngs == sorted(["CP-OFDM-MMSE-64QAM-UNIFORM-BER_vs_SNR.png"] +
                          [f"CP-OFDM-MMSE-64QAM-UNIFORM-SNR{int(s)}_0dB.png" for s in snrs])


def _rr_worker(rank, world, port, tmp, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        M.Simulation.create_from_simulation_settings = classmethod(
            lambda cls, s: [_FakeSim(x) for x in s.signal_noise_ratios])
        os.chdir(tmp)
        runner = M.SimulationRunner(Settings(project_name="P", version="1"), _settings([0.0, 5.0, 10.0, 15.0, 20.0]),
                                    M.ResultsManager(channel_name=f"r{rank}"))
        res = runner.run_all()
        q.put((rank, [r["snr_db"] for r in res]))
    finally:
        dist.destroy_process_group()


def test_runner_round_robin_two_ranks(tmp_path):
    """Reference-stream sweeps under torchrun: SNR points split round-robin, gathered in order."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rr_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    got = dict(q.get(timeout=10) for _ in range(2))
    assert got[0] == got[1] == [0.0, 5.0, 10.0, 15.0, 20.0]


@pytest.mark.gpu
def test_cli_main_on_gpu(tmp_path, monkeypatch):
    """``python -m ofdm_based_systems.main`` on a reduced copy of config/simulation_settings_test.json,
    seeded as the reference's main() was when tests/golden/make_cli_golden.py ran it: the same
    results/ber_results.csv, byte for byte (BER per SNR from the GPU path), plus the image files."""
    import numpy as np
    from numpy.random import PCG64, Generator

    import ofdm_based_systems.bits_generation.models as bg

    want = G["cli_run"]
    monkeypatch.chdir(tmp_path)
    os.makedirs("config/channel_models")
    shutil.copy(os.path.join(ROOT, "config", "settings.json"), "config/settings.json")
    shutil.copy(os.path.join(ROOT, "config", "channel_models", "severe_multipath.npy"), "config/channel_models/")
    cfg = json.load(open(os.path.join(ROOT, "config", "simulation_settings_test.json")))
    cfg["num_symbols"] = want["num_symbols"]
    json.dump(cfg, open("config/simulation_settings.json", "w"))
    defaults = (bg.RandomBitsGenerator.__init__.__defaults__, bg.AdaptiveBitsGenerator.__init__.__defaults__)
    try:
        bg.RandomBitsGenerator.__init__.__defaults__ = (Generator(PCG64(want["seed"])),)
        bg.AdaptiveBitsGenerator.__init__.__defaults__ = (Generator(PCG64(want["seed"])),)
        np.random.seed(want["seed"])
        assert M.main() == want["rc"] == 0
    finally:
        bg.RandomBitsGenerator.__init__.__defaults__, bg.AdaptiveBitsGenerator.__init__.__defaults__ = defaults
    assert open("results/ber_results.csv").read() == want["csv"]
    assert float(want["csv"].splitlines()[1].split(",")[2]) > 0  # a run with errors to compare
    imgs = os.listdir("images/severe_multipath")
    assert len(imgs) == 1 + len(cfg["signal_noise_ratios"]) and any(i.endswith("BER_vs_SNR.png") for i in imgs)
    assert sorted(os.listdir("docs/figures/severe_multipath")) == sorted(imgs)
