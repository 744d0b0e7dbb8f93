"""CLI and results layer: ``python -m ofdm_based_systems.main`` (main.py:1-397 of the reference).

Same classes and behaviour as the reference, on top of the GPU ``Simulation``:

* ``ResultsManager`` (main.py:19-194): the ``results/ber_results.csv`` upsert keyed by
  (simulation_name, snr_db), constellation PNGs named
  ``{prefix}-{modulator}-{eq}-{order}{scheme}-{power}-SNR{snr with '_'}dB.png`` under
  ``images/<channel>/``, the ``...-BER_vs_SNR.png`` semilog plot, and the copy of every
  image into ``docs/figures/<channel>/``.
* ``SimulationRunner`` (main.py:197-344): one ``Simulation`` per SNR point, run in order,
  then plots, CSV and the summary statistics.
* ``main()`` (main.py:347-393): reads ``config/settings.json`` and
  ``config/simulation_settings.json`` from the working directory, names the channel
  directory after the CIR file (CUSTOM), ``flat`` (FLAT) or ``default``, returns 0 / 1.
  The optional command-line flags only override those defaults; with none given the
  behaviour is the reference's.

Under ``torchrun`` every rank runs every SNR point on its own symbol shard (the
simulation all-reduces the counters, ``engine.py``); only rank 0 writes files and prints.
"""

from __future__ import annotations

import argparse
import os
import shutil
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence, Union

import pandas as pd

from ofdm_based_systems.configuration.models import Settings, SimulationSettings
from ofdm_based_systems.simulation.models import Simulation

CSV_COLUMNS = ["simulation_name", "snr_db", "bit_error_rate"]


def _world() -> tuple:
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def _is_rank0() -> bool:
    return _world()[1] == 0


def _say(*args, **kwargs) -> None:
    if _is_rank0():
        print(*args, **kwargs)


def image_stem(prefix_type: str, modulation_type: str, equalization_method: str,
               constellation_order: int, constellation_type: str, power_allocation: str) -> str:
    """Shared filename head of the constellation and BER images (main.py:135-139, 172-176)."""
    return (f"{prefix_type}-{modulation_type}-{equalization_method}-"
            f"{constellation_order}{constellation_type}-{power_allocation}")


def _config_of(result: Dict[str, Any]) -> Dict[str, Any]:
    """The filename fields of a result dict with the reference's fallbacks (main.py:272-278)."""
    return dict(
        prefix_type=result.get("prefix_acronym", "NONE"),
        modulation_type=result.get("modulator_type", "OFDM"),
        equalization_method=result.get("equalizator_type", "NONE"),
        constellation_order=result.get("constellation_order", 16),
        constellation_type=result.get("constellation_scheme", "QAM"),
        power_allocation=result.get("power_allocation_acronym", "UNIFORM"),
    )


class ResultsManager:
    """CSV storage and images of a sweep (main.py:19-194)."""

    def __init__(
        self,
        results_dir: str = "results",
        images_dir: str = "images",
        channel_name: str = "default",
        doc_figures_dir: Union[str, Path, None] = "docs/figures",
    ):
        self.results_dir = Path(results_dir)
        self.channel_name = channel_name
        self.images_dir = Path(images_dir) / channel_name
        self.csv_path = self.results_dir / "ber_results.csv"
        self.doc_figures_dir: Optional[Path] = Path(doc_figures_dir) if doc_figures_dir else None
        self.doc_channel_dir: Optional[Path] = None
        self.results_dir.mkdir(parents=True, exist_ok=True)
        self.images_dir.mkdir(parents=True, exist_ok=True)
        if self.doc_figures_dir:
            self.doc_channel_dir = self.doc_figures_dir / self.channel_name
            self.doc_channel_dir.mkdir(parents=True, exist_ok=True)

    def _mirror_to_docs(self, source_path: Path) -> Optional[Path]:
        """Copy an image below ``docs/figures/<channel>/`` keeping its relative path (main.py:53-67)."""
        if not self.doc_channel_dir or not source_path.exists():
            return None
        try:
            relative: Union[Path, str] = source_path.relative_to(self.images_dir)
        except ValueError:
            relative = source_path.name
        dest = self.doc_channel_dir / relative
        dest.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy2(source_path, dest)
        return dest

    def update_ber_csv(self, simulation_name: str, snr_db: float, bit_error_rate: float) -> None:
        """Upsert one (simulation_name, snr_db) row of ``ber_results.csv`` (main.py:69-101)."""
        if self.csv_path.exists():
            df = pd.read_csv(self.csv_path)
        else:
            df = pd.DataFrame(columns=CSV_COLUMNS)
        hit = (df["simulation_name"] == simulation_name) & (df["snr_db"] == snr_db)
        if hit.any():
            df.loc[hit, "bit_error_rate"] = bit_error_rate
        else:
            row = pd.DataFrame([{"simulation_name": simulation_name, "snr_db": snr_db,
                                 "bit_error_rate": bit_error_rate}])
            df = row if df.empty else pd.concat([df, row], ignore_index=True)
        df.to_csv(self.csv_path, index=False)

    def save_constellation_plot(self, image, prefix_type: str, modulation_type: str,
                                equalization_method: str, constellation_order: int,
                                constellation_type: str, power_allocation: str,
                                snr_db: float) -> Path:
        """Save the PIL constellation image, e.g. ``CP-OFDM-ZF-64QAM-WF-SNR30_0dB.png`` (main.py:103-144)."""
        snr_str = f"{snr_db:.1f}".replace(".", "_")
        stem = image_stem(prefix_type, modulation_type, equalization_method,
                          constellation_order, constellation_type, power_allocation)
        path = self.images_dir / f"{stem}-SNR{snr_str}dB.png"
        image.save(path)
        self._mirror_to_docs(path)
        return path

    def plot_ber_vs_snr(self, results: List[Dict[str, Any]]) -> Path:
        """Semilog BER-vs-SNR plot of a sweep, named after its first result (main.py:146-194)."""
        bers = [r["bit_error_rate"] for r in results if "bit_error_rate" in r]
        snrs = [r["snr_db"] for r in results if "snr_db" in r]
        if not bers or not snrs:
            print("Warning: No BER or SNR data to plot")
            return self.images_dir / "ber_vs_snr.png"
        name = image_stem(**_config_of(results[0])) + "-BER_vs_SNR.png"

        import matplotlib

        matplotlib.use("Agg", force=False)
        import matplotlib.pyplot as plt

        plt.figure(figsize=(10, 6))
        plt.semilogy(snrs, bers, marker="o", linestyle="-", label="BER vs SNR", color="blue")
        plt.xlabel("SNR (dB)", fontsize=12)
        plt.ylabel("Bit Error Rate (BER)", fontsize=12)
        plt.title("BER vs SNR Performance", fontsize=14, fontweight="bold")
        plt.grid(True, which="both", linestyle="--", linewidth=0.5, alpha=0.7)
        plt.legend(fontsize=11)
        plt.tight_layout()
        path = self.images_dir / name
        plt.savefig(path, dpi=150)
        plt.close()
        self._mirror_to_docs(path)
        return path


class SimulationRunner:
    """Runs the SNR sweep of a settings file and hands the results to a ResultsManager (main.py:197-344)."""

    def __init__(self, settings: Settings, simulation_settings: SimulationSettings,
                 results_manager: ResultsManager):
        self.settings = settings
        self.simulation_settings = simulation_settings
        self.results_manager = results_manager

    def run_all(self) -> List[Dict[str, Any]]:
        """One Simulation per SNR value, run in order (main.py:217-249)."""
        _say("=" * 80)
        _say(f"  {self.settings.project_name} v{self.settings.version}")
        _say("=" * 80)
        _say(f"\n{self.simulation_settings}\n")
        simulations = Simulation.create_from_simulation_settings(self.simulation_settings)
        _say(f"Created {len(simulations)} simulation(s) to run\n")
        world, rank = _world()
        if world > 1 and self.simulation_settings.rng_mode == "reference":
            return self._run_round_robin(simulations, world, rank)
        results = []
        for i, sim in enumerate(simulations, start=1):
            if world > 1:  # philox streams: every rank takes a symbol shard of every SNR point
                import torch.distributed as dist

                sim.process_group = dist.group.WORLD
            _say(f"\n{'#' * 80}")
            _say(f"  Running Simulation {i}/{len(simulations)} (SNR = {sim.snr_db} dB)")
            _say(f"{'#' * 80}\n")
            result = sim.run()
            results.append(result)
            _say(f"\n  ✓ Simulation {i} completed")
            _say(f"    BER: {result['bit_error_rate']:.6e}")
            _say(f"    Bit Errors: {result['bit_errors']}/{result['total_bits']}")
            _say(f"    PAPR: {result['papr_db']:.2f} dB")
            if "channel_capacity" in result:
                _say(f"    Channel Capacity: {result.get('channel_capacity', 'N/A')}")
        return results

    def _run_round_robin(self, simulations: List[Simulation], world: int, rank: int) -> List[Dict[str, Any]]:
        """Reference-stream runs draw their bits and noise on the host in sequence, so they are
        not split by symbols: rank r runs SNR points r, r+world, ... whole, and rank 0 gathers
        the results back into sweep order."""
        import torch.distributed as dist

        mine = {}
        for i in range(rank, len(simulations), world):
            print(f"  [rank {rank}] Running Simulation {i + 1}/{len(simulations)} "
                  f"(SNR = {simulations[i].snr_db} dB)")
            mine[i] = simulations[i].run()
        gathered: List[Any] = [None] * world
        dist.all_gather_object(gathered, mine)
        results = [None] * len(simulations)
        for part in gathered:
            for i, r in part.items():
                results[i] = r
        for i, result in enumerate(results, start=1):
            _say(f"\n  ✓ Simulation {i} completed")
            _say(f"    BER: {result['bit_error_rate']:.6e}")
            _say(f"    Bit Errors: {result['bit_errors']}/{result['total_bits']}")
            _say(f"    PAPR: {result['papr_db']:.2f} dB")
        return results

    def process_results(self, results: List[Dict[str, Any]]) -> None:
        """Constellation PNGs, CSV upsert, BER plot and summary (main.py:251-344); rank 0 only."""
        if not _is_rank0():
            return
        if not results:
            print("Warning: No results to process")
            return
        rm = self.results_manager
        print(f"\n{'=' * 80}")
        print("  Processing Results")
        print("=" * 80)

        saved = []
        for result in results:
            if "constellation_plot" in result:
                image = result["constellation_plot"]
                saved.append(rm.save_constellation_plot(image=image, snr_db=result.get("snr_db", 0.0),
                                                        **_config_of(result)))
                image.close()
        print(f"  ✓ Saved {len(saved)} constellation plot(s)")
        if saved and rm.doc_channel_dir:
            print(f"  -> Mirrored constellation plot(s) to {rm.doc_channel_dir}")

        name = results[0].get("title", "unknown").replace(" ", "_")
        for result in results:
            if "bit_error_rate" in result and "snr_db" in result:
                rm.update_ber_csv(simulation_name=name, snr_db=result["snr_db"],
                                  bit_error_rate=result["bit_error_rate"])
        print(f"  ✓ Updated BER results CSV: {rm.csv_path}")

        plot_path = rm.plot_ber_vs_snr(results)
        print(f"  ✓ Generated BER vs SNR plot: {plot_path}")
        if rm.doc_channel_dir:
            print(f"  -> Mirrored BER plot to {rm.doc_channel_dir / plot_path.name}")

        print(f"\n{'=' * 80}")
        print("  Summary Statistics")
        print("=" * 80)
        bers = [r["bit_error_rate"] for r in results]
        snrs = [r["snr_db"] for r in results]
        paprs = [r["papr_db"] for r in results]
        print(f"  SNR Range: {min(snrs):.1f} dB to {max(snrs):.1f} dB")
        print(f"  BER Range: {min(bers):.6e} to {max(bers):.6e}")
        print(f"  Average PAPR: {sum(paprs) / len(paprs):.2f} dB")
        caps = [r.get("channel_capacity") for r in results if "channel_capacity" in r]
        if caps:
            print(f"  Channel Capacity Range: {min(caps):.2f} to {max(caps):.2f} bits/channel use")
        print("=" * 80)


def channel_name_of(simulation_settings: SimulationSettings) -> str:
    """Image subdirectory: the CIR file stem (CUSTOM), ``flat`` (FLAT), else ``default`` (main.py:357-365)."""
    if simulation_settings.channel_type.value == "CUSTOM" and simulation_settings.channel_model_path:
        return Path(simulation_settings.channel_model_path).stem
    if simulation_settings.channel_type.value == "FLAT":
        return "flat"
    return "default"


def _parse(argv: Optional[Sequence[str]]) -> argparse.Namespace:
    p = argparse.ArgumentParser(prog="python -m ofdm_based_systems.main",
                                description="OFDM link simulation sweep on the GPU")
    p.add_argument("--settings", default="config/settings.json")
    p.add_argument("--simulation-settings", default="config/simulation_settings.json")
    p.add_argument("--results-dir", default="results")
    p.add_argument("--images-dir", default="images")
    p.add_argument("--doc-figures-dir", default="docs/figures",
                   help="mirror directory for the images ('' disables it)")
    return p.parse_args([] if argv is None else list(argv))


def _init_distributed() -> None:
    """Join the torchrun process group (one rank per GPU) when launched under torchrun."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return
    import torch
    import torch.distributed as dist

    if dist.is_initialized():
        return
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
    else:
        dist.init_process_group("gloo")


def main(argv: Optional[Sequence[str]] = None) -> int:
    """Entry point (main.py:347-393): 0 on success, 1 on a missing file or a failed run."""
    try:
        args = _parse(argv)
        _init_distributed()
        settings = Settings.from_json(file_path=args.settings)
        simulation_settings = SimulationSettings.from_json(file_path=args.simulation_settings)
        results_manager = ResultsManager(
            results_dir=args.results_dir,
            images_dir=args.images_dir,
            channel_name=channel_name_of(simulation_settings),
            doc_figures_dir=args.doc_figures_dir or None,
        )
        runner = SimulationRunner(settings, simulation_settings, results_manager)
        results = runner.run_all()
        runner.process_results(results)
        _say("\n✓ All simulations completed successfully!\n")
    except FileNotFoundError as e:
        print(f"Error: Configuration file not found - {e}")
        return 1
    except Exception as e:
        print(f"Error during simulation: {e}")
        import traceback

        traceback.print_exc()
        return 1
    return 0


if __name__ == "__main__":
    import sys

    raise SystemExit(main(sys.argv[1:]))
