{{- define "second.labels" -}}
app.kubernetes.io/part-of: scheduler-plugins
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
{{- end -}}
