from mxserve.worker.__main__ import main

if __name__ == "__main__":
    main(dialect="sglang")
