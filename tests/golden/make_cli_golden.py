"""Golden outputs of the reference's results layer (main.py:19-194), numbers and names only.

Run ONLY in the build container, where the reference is importable:

    PYTHONPATH=/root/reference/src PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg \
        python tests/golden/make_cli_golden.py

Drives ``ResultsManager`` in a scratch directory with a fixed sequence of CSV upserts
(new rows, an update of an existing (name, snr) row, a float SNR, a second simulation
name) and saves the CSV text after every step, the file names of the constellation and
BER images it writes (``save_constellation_plot`` / ``plot_ber_vs_snr``) and the files
mirrored under ``docs/figures``; plus ``main()``'s channel-directory naming for each
settings file under ``config/`` and its return code for a missing configuration.
Also runs the reference's ``main()`` end to end on a reduced copy of
``config/simulation_settings_test.json`` (``CLI_NUM_SYMBOLS`` constellation symbols, every SNR
of the file), seeded as make_golden.seed_all does once before ``main()``, and keeps the
``results/ber_results.csv`` it writes (``cli_run``).  Writes ``cli.json``.
"""

from __future__ import annotations

import contextlib
import io
import json
import os
import tempfile

from PIL import Image

OUT = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

UPSERTS = [
    ("CP-OFDM-MMSE", 0.0, 0.25),
    ("CP-OFDM-MMSE", 5.0, 0.125),
    ("CP-OFDM-MMSE", 0.0, 0.2),          # update of an existing row
    ("ZP-SC-OFDM-ZF", 7.5, 1.5e-3),      # second simulation, float SNR
    ("CP-OFDM-MMSE", 10.0, 0.0),
    ("ZP-SC-OFDM-ZF", 7.5, 1.0e-3),      # update again
]

IMAGES = [
    dict(prefix_type="CP", modulation_type="OFDM", equalization_method="ZF", constellation_order=64,
         constellation_type="QAM", power_allocation="WF", snr_db=30.0),
    dict(prefix_type="ZP", modulation_type="SC-OFDM", equalization_method="MMSE", constellation_order=8,
         constellation_type="PSK", power_allocation="UNIFORM", snr_db=12.25),
    dict(prefix_type="NONE", modulation_type="OFDM", equalization_method="NONE", constellation_order=4,
         constellation_type="QAM", power_allocation="UNIFORM", snr_db=-3.0),
]

CLI_NUM_SYMBOLS = 64 * 32
CLI_SEED = 1

BER_RESULTS = [
    {"prefix_acronym": "CP", "modulator_type": "OFDM", "equalizator_type": "MMSE", "constellation_order": 16,
     "constellation_scheme": "QAM", "power_allocation_acronym": "WF", "snr_db": s, "bit_error_rate": b}
    for s, b in ((0.0, 0.1), (10.0, 0.01), (20.0, 0.001))
]


def main() -> None:
    from ofdm_based_systems import main as ref_main
    from ofdm_based_systems.configuration.models import SimulationSettings

    out = {"upserts": [list(u) for u in UPSERTS], "csv_after_step": [], "images": [], "ber_plot": None,
           "mirrored": [], "channel_names": {}}
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        try:
            rm = ref_main.ResultsManager(results_dir="results", images_dir="images", channel_name="severe_multipath")
            for name, snr, ber in UPSERTS:
                rm.update_ber_csv(name, snr, ber)
                with open(rm.csv_path) as fh:
                    out["csv_after_step"].append(fh.read())
            img = Image.new("RGB", (8, 8))
            for kw in IMAGES:
                p = rm.save_constellation_plot(image=img, **kw)
                out["images"].append(os.path.relpath(p, d))
            out["ber_plot"] = os.path.relpath(rm.plot_ber_vs_snr(BER_RESULTS), d)
            out["ber_plot_empty"] = os.path.relpath(rm.plot_ber_vs_snr([]), d)
            for root, _, files in os.walk("docs"):
                out["mirrored"] += sorted(os.path.join(root, f) for f in files)
            out["mirrored"].sort()
            # main() with no configuration in the working directory
            with contextlib.redirect_stdout(io.StringIO()) as buf:
                out["main_missing_config_rc"] = ref_main.main()
            out["main_missing_config_stdout"] = buf.getvalue()
        finally:
            os.chdir(cwd)
    out["cli_run"] = cli_run(ref_main)
    os.chdir(REF)
    try:
        for f in sorted(os.listdir("config")):
            if f.startswith("simulation_settings"):
                s = SimulationSettings.from_json(os.path.join("config", f))
                ch = "default"
                if s.channel_type.value == "CUSTOM" and s.channel_model_path:
                    ch = os.path.splitext(os.path.basename(s.channel_model_path))[0]
                elif s.channel_type.value == "FLAT":
                    ch = "flat"
                out["channel_names"][f] = ch
    finally:
        os.chdir(cwd)
    with open(os.path.join(OUT, "cli.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote cli.json")


def cli_run(ref_main) -> dict:
    """The reference's main() on the reduced test configuration, seeded once before the run:
    the CSV of BER per SNR it writes."""
    import shutil

    import numpy as np
    from numpy.random import PCG64, Generator

    import ofdm_based_systems.bits_generation.models as bg

    cfg = json.load(open(os.path.join(REF, "config", "simulation_settings_test.json")))
    cfg["num_symbols"] = CLI_NUM_SYMBOLS
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        try:
            os.makedirs("config/channel_models")
            shutil.copy(os.path.join(REF, "config", "settings.json"), "config/settings.json")
            shutil.copy(os.path.join(REF, "config", "channel_models", "severe_multipath.npy"), "config/channel_models/")
            json.dump(cfg, open("config/simulation_settings.json", "w"))
            bg.RandomBitsGenerator.__init__.__defaults__ = (Generator(PCG64(CLI_SEED)),)
            bg.AdaptiveBitsGenerator.__init__.__defaults__ = (Generator(PCG64(CLI_SEED)),)
            np.random.seed(CLI_SEED)
            with contextlib.redirect_stdout(io.StringIO()):
                rc = ref_main.main()
            csv = open("results/ber_results.csv").read()
        finally:
            os.chdir(cwd)
    return {"num_symbols": CLI_NUM_SYMBOLS, "seed": CLI_SEED, "rc": rc, "csv": csv}


if __name__ == "__main__":
    main()
