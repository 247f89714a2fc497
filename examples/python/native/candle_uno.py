"""candle_uno (reference examples/cpp/candle_uno, examples/python/native): zoo model "candle_uno" trained on
synthetic batches through FFModel; flags in zoo.py."""
from zoo import run

if __name__ == "__main__":
    run("candle_uno")
