"""Teacher -> student weight transfer shared by the *_net2net examples (reference
examples/python/keras/*_net2net.py): train a teacher, read each layer's weights with
layer.get_weights(ffmodel), build a student with the same layer shapes, write them with
layer.set_weights(ffmodel, kernel, bias), and keep training the student."""
import numpy as np


def transfer(teacher_layers, teacher_model, student_layers, student_model):
    for t, s in zip(teacher_layers, student_layers):
        ws = t.get_weights(teacher_model.ffmodel)
        s.set_weights(student_model.ffmodel, *ws)
        got = s.get_weights(student_model.ffmodel)
        assert all(np.allclose(a, b) for a, b in zip(ws, got)), f"weights of {s.name} did not transfer"
