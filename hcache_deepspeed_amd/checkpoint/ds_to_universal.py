"""``deepspeed.checkpoint.ds_to_universal`` import path and CLI (reference checkpoint/ds_to_universal.py:50,469)::

    python -m hcache_deepspeed_amd.checkpoint.ds_to_universal --input_folder ckpt/global_step10 \
        --output_folder ckpt/global_step10_universal
"""
import argparse

from .universal import ds_to_universal  # noqa: F401


def parse_arguments(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--input_folder", required=True, help="ZeRO checkpoint folder (a tag directory or its parent)")
    ap.add_argument("--output_folder", required=True, help="universal checkpoint output folder")
    ap.add_argument("--tag", default=None)
    ap.add_argument("--num_extract_workers", type=int, default=4,
                    help="processes extracting ZeRO shards (one job per state and TP rank)")
    ap.add_argument("--num_merge_workers", type=int, default=2,
                    help="processes merging TP slices (one job per state and parameter; memory-heavier)")
    ap.add_argument("--keep_temp_folder", action="store_true", help="keep <output>/tmp (the extracted slices)")
    ap.add_argument("--no_strict", dest="strict", action="store_false",
                    help="warn instead of failing when a parameter did not convert cleanly")
    ap.add_argument("--inject_missing_state", action="store_true",
                    help="supply a default universal_checkpoint_info to a source that lacks it")
    return ap.parse_args(argv)


def main(args):
    print(f"Converting DeepSpeed checkpoint in {args.input_folder} to Universal checkpoint in {args.output_folder}")
    ds_to_universal(args.input_folder, args.output_folder, tag=args.tag, num_extract_workers=args.num_extract_workers,
                    num_merge_workers=args.num_merge_workers, keep_temp_folder=args.keep_temp_folder,
                    strict=args.strict, inject_missing_state=args.inject_missing_state)


if __name__ == "__main__":
    main(parse_arguments())
